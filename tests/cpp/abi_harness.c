/*
 * abi_harness.c — a plain C client of libl7match.so (no ctypes, no torch):
 * the binding a cgo shim or an Envoy filter would use.
 *
 *   abi_harness <rules.txt> <requests.bin> <threads> <iters> <out.bin> [batcher]
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
 *
 * With the 6th argument `batcher`: the call-site shape instead.  One
 * l7m_batcher over the handle; `threads` host threads each take every
 * threads-th request and decide it with the blocking per-request
 * l7m_batcher_eval (canAccess / decodeHeaders), while thread 0 swaps in a
 * second compile of the same rules halfway (l7m_batcher_set_ruleset, the
 * policy update).  Every denied request gets its 403 body
 * (l7m_http_deny_body).  out.bin: i32 verdicts[n] by request index, then
 * u64 {batches, requests, denied, forwarded} (l7m_batcher_stats and
 * l7m_proxy_stats_add over the verdicts).
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

typedef struct {
  l7m_batcher* b;
  l7m_ruleset* swap_to;  /* thread 0 only */
  const uint8_t* arena;
  const uint64_t* offs;
  size_t n, arena_bytes;
  int t, threads;
  int32_t* verdicts;
  int rc;
} bjob_t;

static void* run_batched(void* arg) {
  bjob_t* j = (bjob_t*)arg;
  char body[64];
  for (size_t i = (size_t)j->t; i < j->n && j->rc == L7M_OK; i += (size_t)j->threads) {
    if (j->swap_to && i >= j->n / 2) {
      j->rc = l7m_batcher_set_ruleset(j->b, j->swap_to);
      j->swap_to = NULL;
      if (j->rc != L7M_OK) break;
    }
    const size_t end = i + 1 < j->n ? j->offs[i + 1] : j->arena_bytes;
    j->rc = l7m_batcher_eval(j->b, j->arena + j->offs[i], (size_t)(end - j->offs[i]), &j->verdicts[i]);
    if (j->rc == L7M_OK && j->verdicts[i] == L7M_VERDICT_DENY &&
        l7m_http_deny_body("", body, sizeof body) != strlen("Access denied\r\n"))
      j->rc = -100;
  }
  return NULL;
}

static int batched(l7m_ruleset* rs, l7m_ruleset* rs2, const uint8_t* arena, size_t ab, const uint64_t* offs,
                   size_t n, int threads, const char* out) {
  l7m_batcher* b = NULL;
  l7m_batcher_opts o;
  memset(&o, 0, sizeof o);
  o.struct_size = sizeof o;
  o.max_delay_us = 500;
  if (l7m_batcher_create(rs, &o, &b) != L7M_OK) return 8;
  int32_t* verd = (int32_t*)malloc(n * 4);
  bjob_t* jobs = (bjob_t*)calloc((size_t)threads, sizeof(bjob_t));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (bjob_t){b, t == 0 ? rs2 : NULL, arena, offs, n, ab, t, threads, verd, L7M_OK};
    pthread_create(&th[t], NULL, run_batched, &jobs[t]);
  }
  int bad = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    if (jobs[t].rc != L7M_OK) {
      fprintf(stderr, "thread %d: batcher %d\n", t, jobs[t].rc);
      bad = 1;
    }
  }
  uint64_t st[4] = {0, 0, 0, 0};
  l7m_batcher_stats(b, &st[0], &st[1]);
  l7m_batcher_destroy(b);
  l7m_proxy_stats ps;
  memset(&ps, 0, sizeof ps);
  if (l7m_proxy_stats_add(verd, n, &ps) != L7M_OK) bad = 1;
  st[2] = ps.denied;
  st[3] = ps.forwarded;
  FILE* f = fopen(out, "wb");
  if (!f) return 7;
  fwrite(verd, 4, n, f);
  fwrite(st, 8, 4, f);
  fclose(f);
  printf("abi_harness: batcher, %zu requests, %d threads, %llu batches: %s\n", n, threads,
         (unsigned long long)st[0], bad ? "FAILED" : "ok");
  return bad;
}

static char* dup_range(const char* a, const char* b) {
  char* s = (char*)malloc((size_t)(b - a) + 1);
  memcpy(s, a, (size_t)(b - a));
  s[b - a] = 0;
  return s;
}

int main(int argc, char** argv) {
  if (argc != 6 && !(argc == 7 && strcmp(argv[6], "batcher") == 0)) {
    fprintf(stderr, "usage: %s rules.txt requests.bin threads iters out.bin [batcher]\n", argv[0]);
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
  if (argc == 7) {
    l7m_ruleset* rs2 = NULL;
    if (l7m_compile_http(rules, nr, NULL, &rs2, err, sizeof err) != L7M_OK) return 5;
    const int r = batched(rs, rs2, arena, ab, offs, n, threads, argv[5]);
    l7m_release(rs2);
    l7m_release(rs);
    return r;
  }
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
