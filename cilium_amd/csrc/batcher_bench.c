/* batcher_bench.c — call-site measurement of the drop-in path (SURVEY.md
 * §8(d) "end-to-end"): T caller threads each decide one request at a time with
 * the blocking l7m_batcher_eval, the call shape of canAccess
 * (pkg/proxy/kafka.go:116-152) and AccessFilter::decodeHeaders
 * (envoy/cilium_l7policy.cc:126-186).  Plain C client of libl7match.so; the
 * workload comes from libl7gen.so (the bench generator).
 *
 *   batcher_bench <config 2|3> <n_requests> <seconds> <eager 0|1> <threads>...
 *
 * Prints one JSON object per thread count: verdicts/s, per-call latency
 * percentiles (us), batches, mean batch size, and mismatches against one
 * l7m_eval of the same records (must be 0). */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/l7match.h"

typedef uint64_t (*gen_fn)(int, uint64_t, uint32_t, uint64_t, uint64_t, uint8_t*, uint64_t, uint64_t*, int);
typedef const char* (*rules_fn)(int, uint64_t, uint32_t);

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static l7m_batcher* g_b;
static const uint8_t* g_arena;
static const uint64_t* g_offs;
static const int32_t* g_expect;
static uint64_t g_n, g_arena_bytes;
static double g_end;
static int g_threads;

typedef struct {
  int t;
  uint64_t done, bad;
  float* lat;  /* us */
  uint64_t cap;
} Arg;

static void* worker(void* p) {
  Arg* a = (Arg*)p;
  uint64_t i = (uint64_t)a->t * 7919u % g_n;
  while (now_s() < g_end && a->done < a->cap) {
    const uint64_t o = g_offs[i], e = i + 1 < g_n ? g_offs[i + 1] : g_arena_bytes;
    int32_t v = 0;
    const double t0 = now_s();
    if (l7m_batcher_eval(g_b, g_arena + o, (size_t)(e - o), &v) != L7M_OK) {
      a->bad++;
      break;
    }
    a->lat[a->done++] = (float)((now_s() - t0) * 1e6);
    if (v != g_expect[i]) a->bad++;
    i += (uint64_t)g_threads;
    if (i >= g_n) i -= g_n;
  }
  return NULL;
}

/* cgroup v2 CPU throttling counters (/sys/fs/cgroup/cpu.stat), -1 if absent */
static void cpu_stat(long long* nr_throttled, long long* throttled_usec) {
  *nr_throttled = *throttled_usec = -1;
  FILE* f = fopen("/sys/fs/cgroup/cpu.stat", "r");
  if (!f) return;
  char k[64];
  long long v;
  while (fscanf(f, "%63s %lld", k, &v) == 2) {
    if (!strcmp(k, "nr_throttled")) *nr_throttled = v;
    if (!strcmp(k, "throttled_usec")) *throttled_usec = v;
  }
  fclose(f);
}

static int cmpf(const void* x, const void* y) {
  const float a = *(const float*)x, b = *(const float*)y;
  return a < b ? -1 : a > b;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s config n seconds eager threads...\n", argv[0]);
    return 2;
  }
  const int cfg = atoi(argv[1]);
  const uint64_t n = strtoull(argv[2], 0, 10);
  const double secs = atof(argv[3]);
  const int eager = atoi(argv[4]);
  char path[4096];
  snprintf(path, sizeof path, "%s", argv[0]);
  char* slash = strrchr(path, '/');
  if (slash) slash[1] = 0; else strcpy(path, "./");
  strcat(path, "libl7gen.so");
  void* gen = dlopen(path, RTLD_NOW);
  if (!gen) {
    fprintf(stderr, "dlopen %s: %s\n", path, dlerror());
    return 2;
  }
  gen_fn gen_requests = (gen_fn)dlsym(gen, "l7g_requests");
  rules_fn gen_rules = (rules_fn)dlsym(gen, "l7g_rules_text");
  const uint64_t seed = cfg == 2 ? 0xC2 : 0xC3;
  const uint32_t n_rules = cfg == 2 ? 1000 : 10000;
  /* rules: one per line, \t-separated fields (cilium_amd/workloads.py) */
  char* text = strdup(gen_rules(cfg, seed, n_rules));
  l7m_http_rule* hr = calloc(n_rules, sizeof *hr);
  l7m_kafka_rule* kr = calloc(n_rules, sizeof *kr);
  char*** hdrs = calloc(n_rules, sizeof *hdrs);
  uint32_t r = 0;
  for (char* line = strtok(text, "\n"); line && r < n_rules; line = strtok(NULL, "\n"), ++r) {
    char* f[6] = {0};
    int k = 0;
    for (char* q = line; k < 6; ++k) {
      f[k] = q;
      char* tab = strchr(q, '\t');
      if (!tab) { ++k; break; }
      *tab = 0;
      q = tab + 1;
    }
    for (int j = 0; j < 6; ++j)
      if (f[j] && !*f[j]) f[j] = NULL;
    if (cfg == 2) {
      hr[r].path = f[0];
      hr[r].method = f[1];
      hr[r].host = f[2];
      hdrs[r] = calloc(8, sizeof(char*));
      uint32_t nh = 0;
      for (char* h = f[3]; h && *h && nh < 8;) {
        hdrs[r][nh++] = h;
        char* us = strchr(h, '\x1f');
        if (!us) break;
        *us = 0;
        h = us + 1;
      }
      hr[r].headers = (const char* const*)hdrs[r];
      hr[r].n_headers = nh;
    } else {
      kr[r].role = f[0];
      kr[r].api_key = f[1];
      kr[r].api_version = f[2];
      kr[r].client_id = f[3];
      kr[r].topic = f[4];
    }
  }
  l7m_ruleset* rs = NULL;
  char err[512];
  int rc = cfg == 2 ? l7m_compile_http(hr, r, NULL, &rs, err, sizeof err)
                    : l7m_compile_kafka(kr, r, NULL, &rs, err, sizeof err);
  if (rc) {
    fprintf(stderr, "compile: %d %s\n", rc, err);
    return 1;
  }
  const uint64_t bytes = gen_requests(cfg, seed, n_rules, 0, n, NULL, 0, NULL, 16);
  uint8_t* arena = calloc(bytes + 64, 1);
  uint64_t* offs = malloc(n * 8);
  gen_requests(cfg, seed, n_rules, 0, n, arena, bytes + 64, offs, 16);
  int32_t* expect = malloc(n * 4);
  if ((rc = l7m_eval(rs, arena, bytes, offs, n, expect, NULL, 0))) {
    fprintf(stderr, "eval: %d\n", rc);
    return 1;
  }
  g_arena = arena;
  g_offs = offs;
  g_expect = expect;
  g_n = n;
  g_arena_bytes = bytes;
  for (int a = 5; a < argc; ++a) {
    const int T = atoi(argv[a]);
    l7m_batcher_opts o;
    memset(&o, 0, sizeof o);
    o.struct_size = sizeof o;
    o.max_batch = 65536;
    o.max_delay_us = 200;
    o.in_flight = getenv("L7M_IN_FLIGHT") ? (uint32_t)atoi(getenv("L7M_IN_FLIGHT")) : 0;  /* 0: the library default (4) */
    o.eager = (uint32_t)eager;
    if ((rc = l7m_batcher_create(rs, &o, &g_b))) return 1;
    g_threads = T;
    Arg* args = calloc(T, sizeof *args);
    pthread_t* th = calloc(T, sizeof *th);
    const uint64_t cap = 4000000 / T + 1000;
    uint64_t b0 = 0, r0 = 0;
    l7m_batcher_stats(g_b, &b0, &r0);
    long long thr0, thu0, thr1, thu1;
    cpu_stat(&thr0, &thu0);
    const double t0 = now_s();
    g_end = t0 + secs;
    for (int t = 0; t < T; ++t) {
      args[t].t = t;
      args[t].cap = cap;
      args[t].lat = malloc(cap * sizeof(float));
      pthread_create(&th[t], NULL, worker, &args[t]);
    }
    uint64_t done = 0, bad = 0;
    for (int t = 0; t < T; ++t) {
      pthread_join(th[t], NULL);
      done += args[t].done;
      bad += args[t].bad;
    }
    const double dt = now_s() - t0;
    cpu_stat(&thr1, &thu1);
    uint64_t b1 = 0, r1 = 0;
    l7m_batcher_stats(g_b, &b1, &r1);
    l7m_batcher_profile pf;
    memset(&pf, 0, sizeof pf);
    l7m_batcher_get_profile(g_b, &pf);
    float* all = malloc((done ? done : 1) * sizeof(float));
    uint64_t k = 0;
    for (int t = 0; t < T; ++t) {
      memcpy(all + k, args[t].lat, args[t].done * sizeof(float));
      k += args[t].done;
      free(args[t].lat);
    }
    qsort(all, done, sizeof(float), cmpf);
    printf("{\"threads\": %d, \"in_flight\": %u, \"eager\": %d, \"verdicts_per_s\": %.1f, \"p50_us\": %.1f, \"p99_us\": %.1f, "
           "\"max_us\": %.1f, \"batches\": %llu, \"mean_batch\": %.1f, \"requests\": %llu, \"mismatches\": %llu, "
           "\"phases_us\": {\"fill\": %.2f, \"launch\": %.2f, \"gpu\": %.2f, \"wake\": %.2f}, "
           "\"resident\": {\"batches\": %llu, \"rounds\": %llu, \"read_us\": %.2f, \"eval_us\": %.2f, \"sync_us\": %.2f}, "
           "\"cgroup_nr_throttled\": %lld, \"cgroup_throttled_usec\": %lld}\n",
           T, o.in_flight, eager, done / dt, done ? all[done / 2] : 0.0, done ? all[(uint64_t)(done * 0.99)] : 0.0,
           done ? all[done - 1] : 0.0, (unsigned long long)(b1 - b0),
           (b1 - b0) ? (double)(r1 - r0) / (double)(b1 - b0) : 0.0, (unsigned long long)done,
           (unsigned long long)bad, pf.fill_us, pf.launch_us, pf.gpu_us, pf.wake_us,
           (unsigned long long)pf.resident_batches, (unsigned long long)pf.resident_rounds, pf.resident_read_us, pf.resident_eval_us, pf.resident_sync_us,
           thr0 >= 0 ? thr1 - thr0 : -1, thu0 >= 0 ? thu1 - thu0 : -1);
    fflush(stdout);
    free(all);
    free(args);
    free(th);
    l7m_batcher_destroy(g_b);
  }
  l7m_release(rs);
  return 0;
}
