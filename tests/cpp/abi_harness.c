/*
 * abi_harness.c — a plain C client of libl7match.so (no ctypes, no torch):
 * the binding a cgo shim or an Envoy filter would use.
 *
 *   abi_harness <rules.txt> <requests.bin> <threads> <iters> <out.bin>
 *
 * rules.txt    one HTTP rule per line: path \t method \t host \t headers (\x1f-separated)
 * requests.bin u64 n, u64 arena_bytes, u64 offsets[n], arena bytes
 * out.bin      i32 verdicts[n] of thread 0, then u64 rule_hits[n_rules + 2] summed
 *              over every call of every thread
 *
 * Compiles the rules once (l7m_compile_http), then `threads` host threads each
 * call l7m_eval `iters` times concurrently on the SAME handle (the reentrancy
 * promise of include/l7match.h) and compare their verdicts with thread 0's.
 * Exit status 0 = every call succeeded and every thread saw identical verdicts.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/l7match.h"

typedef struct {
  const l7m_ruleset* rs;
  const uint8_t* arena;
  size_t arena_bytes;
  const uint64_t* offs;
  size_t n;
  int iters;
  int32_t* verdicts;
  uint64_t* hits;
  size_t n_ctr;
  int rc;
} job_t;

static void* run(void* arg) {
  job_t* j = (job_t*)arg;
  for (int it = 0; it < j->iters && j->rc == L7M_OK; ++it)
    j->rc = l7m_eval(j->rs, j->arena, j->arena_bytes, j->offs, j->n, j->verdicts, j->hits, 0);
  return NULL;
}

static char* dup_range(const char* a, const char* b) {
  char* s = (char*)malloc((size_t)(b - a) + 1);
  memcpy(s, a, (size_t)(b - a));
  s[b - a] = 0;
  return s;
}

int main(int argc, char** argv) {
  if (argc != 6) {
    fprintf(stderr, "usage: %s rules.txt requests.bin threads iters out.bin\n", argv[0]);
    return 2;
  }
  const int threads = atoi(argv[3]), iters = atoi(argv[4]);
  if (l7m_abi_version() != L7M_ABI_VERSION) {
    fprintf(stderr, "ABI mismatch: library %d, header %d\n", l7m_abi_version(), L7M_ABI_VERSION);
    return 3;
  }
  /* ---- rules ---- */
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 4;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  char* text = (char*)malloc((size_t)sz + 1);
  if (fread(text, 1, (size_t)sz, f) != (size_t)sz) return 4;
  text[sz] = 0;
  fclose(f);
  size_t cap = 1024, nr = 0;
  l7m_http_rule* rules = (l7m_http_rule*)calloc(cap, sizeof(l7m_http_rule));
  for (char* line = text; *line;) {
    char* eol = strchr(line, '\n');
    if (!eol) eol = line + strlen(line);
    char* fld[4] = {0, 0, 0, 0};
    char* p = line;
    for (int k = 0; k < 4; ++k) {
      char* e = k < 3 ? memchr(p, '\t', (size_t)(eol - p)) : eol;
      if (!e) e = eol;
      fld[k] = dup_range(p, e);
      p = e < eol ? e + 1 : eol;
    }
    if (nr == cap) {
      cap *= 2;
      rules = (l7m_http_rule*)realloc(rules, cap * sizeof(l7m_http_rule));
    }
    l7m_http_rule* r = &rules[nr++];
    memset(r, 0, sizeof *r);
    r->path = fld[0];
    r->method = fld[1];
    r->host = fld[2];
    if (fld[3][0]) {
      const char** hs = (const char**)calloc(64, sizeof(char*));
      uint32_t nh = 0;
      for (char* h = fld[3]; h && nh < 64;) {
        char* e = strchr(h, '\x1f');
        hs[nh++] = e ? dup_range(h, e) : h;
        h = e ? e + 1 : NULL;
      }
      r->headers = hs;
      r->n_headers = nh;
    }
    line = *eol ? eol + 1 : eol;
  }
  char err[512];
  l7m_ruleset* rs = NULL;
  int rc = l7m_compile_http(rules, nr, NULL, &rs, err, sizeof err);
  if (rc != L7M_OK) {
    fprintf(stderr, "compile: %d %s\n", rc, err);
    return 5;
  }
  l7m_ruleset_info info;
  l7m_ruleset_get_info(rs, &info);
  /* ---- requests ---- */
  f = fopen(argv[2], "rb");
  if (!f) return 6;
  uint64_t hdr[2];
  if (fread(hdr, 8, 2, f) != 2) return 6;
  const size_t n = (size_t)hdr[0], ab = (size_t)hdr[1];
  uint64_t* offs = (uint64_t*)malloc(n * 8);
  uint8_t* arena = (uint8_t*)malloc(ab);
  if (fread(offs, 8, n, f) != n || fread(arena, 1, ab, f) != ab) return 6;
  fclose(f);
  /* ---- concurrent evaluation on one handle ---- */
  job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (job_t){rs, arena, ab, offs, n, iters, (int32_t*)malloc(n * 4),
                      (uint64_t*)calloc(info.n_counters, 8), info.n_counters, L7M_OK};
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  int bad = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    if (jobs[t].rc != L7M_OK) {
      fprintf(stderr, "thread %d: l7m_eval %d\n", t, jobs[t].rc);
      bad = 1;
    }
  }
  uint64_t* sum = (uint64_t*)calloc(info.n_counters, 8);
  for (int t = 0; t < threads && !bad; ++t) {
    if (memcmp(jobs[t].verdicts, jobs[0].verdicts, n * 4) != 0) {
      fprintf(stderr, "thread %d verdicts differ from thread 0\n", t);
      bad = 1;
    }
    for (size_t i = 0; i < info.n_counters; ++i) sum[i] += jobs[t].hits[i];
  }
  f = fopen(argv[5], "wb");
  if (!f) return 7;
  fwrite(jobs[0].verdicts, 4, n, f);
  fwrite(sum, 8, info.n_counters, f);
  fclose(f);
  l7m_release(rs);
  printf("abi_harness: %zu rules, %zu requests, %d threads x %d calls: %s\n", nr, n, threads, iters,
         bad ? "FAILED" : "ok");
  return bad;
}
