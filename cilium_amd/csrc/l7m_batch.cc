// l7m_batch.cc — the batching front-end of the verdict path (l7m_batcher in
// include/l7match.h).
//
// The reference decides one request per call on the connection's own
// goroutine / Envoy worker: canAccess -> MatchesRule (pkg/proxy/kafka.go:116-152,
// called from handleRequest :232-306) and AccessFilter::decodeHeaders ->
// NetworkPolicyMap::Allowed (envoy/cilium_l7policy.cc:126-186).  A GPU call
// per request would cost more than the verdict, so the batcher keeps that
// per-request, blocking call shape while many callers' requests share one
// l7m_eval: a caller appends its record to the batch being filled and waits;
// a flusher evaluates the batch when it holds max_batch requests or its first
// request has waited max_delay_us, while the next batch fills.
//
// Pipelining: `in_flight` flusher threads (default 2) each take the next
// ready batch (with `eager`, as soon as a flusher is free: batches then grow
// with the load instead of waiting for max_delay_us), so batch k+1's H2D copy runs while batch k's kernel and D2H
// run (l7m_eval is reentrant: every call has its own stream and device
// buffers).  Batches live in pinned host memory (recycled, never freed while
// the batcher lives), so the copies are DMA transfers, not staged.
// l7m_batcher_set_ruleset is the policy update (Redirect.updateRules,
// pkg/proxy/redirect.go:68-74): batches flushed afterwards use the new rules.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstddef>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/l7match.h"

namespace {

using Clock = std::chrono::steady_clock;

// Growable pinned host buffer (hipHostMalloc); grows by doubling.
template <class T>
struct PinnedVec {
  T* p = nullptr;
  size_t n = 0, cap = 0;
  PinnedVec() = default;
  PinnedVec(const PinnedVec&) = delete;
  PinnedVec& operator=(const PinnedVec&) = delete;
  ~PinnedVec() {
    if (p) (void)hipHostFree(p);
  }
  bool reserve(size_t want) {
    if (want <= cap) return true;
    size_t c = cap ? cap : 1024;
    while (c < want) c *= 2;
    void* q = nullptr;
    if (hipHostMalloc(&q, c * sizeof(T), hipHostMallocDefault) != hipSuccess) return false;
    if (n) std::memcpy(q, p, n * sizeof(T));
    if (p) (void)hipHostFree(p);
    p = static_cast<T*>(q);
    cap = c;
    return true;
  }
};

// A batch's completion has its own mutex / condition variable, so finishing
// one batch wakes only its callers (no thundering herd across batches) and
// they do not contend with callers appending to the next batch.
struct Batch {
  PinnedVec<uint8_t> arena;
  PinnedVec<uint64_t> offs;
  PinnedVec<uint32_t> ids;  // source identities (Kafka rule sets)
  PinnedVec<int32_t> verd;
  Clock::time_point first;
  std::mutex m;             // guards done, rc, waiters
  std::condition_variable cv;
  bool done = false;
  int rc = L7M_OK;
  uint32_t waiters = 0;  // callers that have not read their verdict yet
  void reset() {
    arena.n = offs.n = ids.n = verd.n = 0;
    done = false;
    rc = L7M_OK;
    waiters = 0;
  }
};

}  // namespace

struct l7m_batcher {
  std::mutex mu;  // guards cur, pool, rs, stop, stats (lock order: mu, then a batch's m)
  std::condition_variable cv_flush, cv_idle;
  l7m_ruleset* rs = nullptr;
  uint32_t max_batch = 65536;
  uint32_t max_delay_us = 200;
  uint32_t in_flight = 2;
  bool eager = false;  // flush as soon as a flusher is free (no deadline wait)
  int device = 0;
  Batch* cur = nullptr;
  std::vector<Batch*> pool;     // recycled batches (pinned buffers kept)
  std::vector<Batch*> all;      // every batch ever made (freed at destroy)
  bool stop = false;
  std::atomic<uint32_t> callers{0};  // threads inside eval()
  uint64_t batches = 0, requests = 0;
  std::vector<std::thread> flushers;

  Batch* fresh() {  // under mu
    Batch* b;
    if (!pool.empty()) {
      b = pool.back();
      pool.pop_back();
    } else {
      b = new Batch();
      all.push_back(b);
    }
    b->reset();
    return b;
  }

  void run() {
    (void)hipSetDevice(device);
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      while (!stop && cur->offs.n == 0) cv_flush.wait(lk);
      if (cur->offs.n == 0 && stop) return;
      // full, or the first request has waited long enough (or shutting down)
      Batch* const b = cur;
      const auto deadline = b->first + std::chrono::microseconds(max_delay_us);
      while (!eager && !stop && cur == b && b->offs.n < max_batch && Clock::now() < deadline)
        cv_flush.wait_until(lk, deadline);
      if (cur != b) continue;  // another flusher took it
      cur = fresh();
      l7m_ruleset* r = rs;
      l7m_retain(r);
      ++batches;
      requests += b->offs.n;
      lk.unlock();
      cv_flush.notify_one();  // a second flusher may start on the next batch
      int rc = b->verd.reserve(b->offs.n) ? L7M_OK : L7M_ENOMEM;
      if (rc == L7M_OK) {
        l7m_ruleset_info info;
        l7m_ruleset_get_info(r, &info);
        rc = l7m_eval_ids(r, b->arena.p, b->arena.n, b->offs.p, b->offs.n,
                          info.proto == L7M_PROTO_KAFKA ? b->ids.p : nullptr, b->verd.p, nullptr, 0);
      }
      l7m_release(r);
      {
        std::lock_guard<std::mutex> g(b->m);
        b->rc = rc;
        b->done = true;
      }
      b->cv.notify_all();
      lk.lock();
    }
  }

  int eval(const uint8_t* rec, size_t len, uint32_t src_identity, int32_t* verdict) {
    std::unique_lock<std::mutex> lk(mu);
    if (stop) return L7M_EINVAL;
    Batch* b = cur;
    const size_t idx = b->offs.n;
    const size_t off = b->arena.n, padded = (len + 3) & ~size_t(3);
    // + 64 bytes of zero tail for the kernels' aligned loads (l7m_eval pads its copy too)
    if (!b->arena.reserve(off + padded + 64) || !b->offs.reserve(idx + 1) || !b->ids.reserve(idx + 1))
      return L7M_ENOMEM;
    callers.fetch_add(1);
    if (idx == 0) b->first = Clock::now();
    b->offs.p[idx] = off;
    b->ids.p[idx] = src_identity;
    if (len) std::memcpy(b->arena.p + off, rec, len);
    std::memset(b->arena.p + off + len, 0, padded - len);
    b->arena.n = off + padded;
    b->offs.n = idx + 1;
    {
      std::lock_guard<std::mutex> g(b->m);  // b is not in flight yet: done is false
      ++b->waiters;
    }
    if (idx == 0 || b->offs.n >= max_batch) cv_flush.notify_one();
    lk.unlock();
    int rc;
    bool last;
    {
      std::unique_lock<std::mutex> bl(b->m);
      b->cv.wait(bl, [&] { return b->done; });
      rc = b->rc;
      if (rc == L7M_OK) *verdict = b->verd.p[idx];
      last = --b->waiters == 0;
    }
    if (last) {  // the last reader recycles the batch
      lk.lock();
      pool.push_back(b);
      lk.unlock();
    }
    if (callers.fetch_sub(1) == 1) {
      std::lock_guard<std::mutex> g(mu);
      cv_idle.notify_all();
    }
    return rc;
  }
};

extern "C" {

int l7m_batcher_create(l7m_ruleset* rs, const l7m_batcher_opts* opts, l7m_batcher** out) {
  if (!rs || !out) return L7M_EINVAL;
  auto* b = new (std::nothrow) l7m_batcher();
  if (!b) return L7M_ENOMEM;
  if (opts) {
    l7m_batcher_opts o{};
    const size_t k = opts->struct_size == 0 || opts->struct_size > sizeof o ? sizeof o : opts->struct_size;
    std::memcpy(&o, opts, k);
    if (o.max_batch) b->max_batch = o.max_batch;
    if (o.max_delay_us) b->max_delay_us = o.max_delay_us;
    if (k >= offsetof(l7m_batcher_opts, in_flight) + sizeof o.in_flight && o.in_flight)
      b->in_flight = o.in_flight > 8 ? 8 : o.in_flight;
    if (k >= offsetof(l7m_batcher_opts, eager) + sizeof o.eager) b->eager = o.eager != 0;
    b->device = o.device;
  }
  b->cur = b->fresh();
  l7m_retain(rs);
  b->rs = rs;
  for (uint32_t i = 0; i < b->in_flight; ++i) b->flushers.emplace_back([b] { b->run(); });
  *out = b;
  return L7M_OK;
}

int l7m_batcher_set_ruleset(l7m_batcher* b, l7m_ruleset* rs) {
  if (!b || !rs) return L7M_EINVAL;
  l7m_retain(rs);
  l7m_ruleset* old;
  {
    std::lock_guard<std::mutex> lk(b->mu);
    old = b->rs;
    b->rs = rs;
  }
  l7m_release(old);
  return L7M_OK;
}

int l7m_batcher_eval(l7m_batcher* b, const uint8_t* rec, size_t len, int32_t* verdict) {
  if (!b || (!rec && len) || !verdict) return L7M_EINVAL;
  return b->eval(rec, len, 0, verdict);
}

int l7m_batcher_eval_from(l7m_batcher* b, const uint8_t* rec, size_t len, uint32_t src_identity, int32_t* verdict) {
  if (!b || (!rec && len) || !verdict) return L7M_EINVAL;
  return b->eval(rec, len, src_identity, verdict);
}

int l7m_batcher_eval_http(l7m_batcher* b, const l7m_http_request* req, int32_t* verdict) {
  if (!b || !req || !verdict) return L7M_EINVAL;
  const size_t sz = l7m_http_record_size(req);
  if (!sz) return L7M_EINVAL;
  std::vector<uint8_t> rec(sz);
  uint64_t off = 0;
  if (l7m_pack_http(req, 1, rec.data(), rec.size(), &off) != sz) return L7M_EINVAL;
  return b->eval(rec.data(), rec.size(), 0, verdict);
}

int l7m_batcher_stats(l7m_batcher* b, uint64_t* batches, uint64_t* requests) {
  if (!b) return L7M_EINVAL;
  std::lock_guard<std::mutex> lk(b->mu);
  if (batches) *batches = b->batches;
  if (requests) *requests = b->requests;
  return L7M_OK;
}

// Safe with calls in flight: pending batches are still evaluated, new calls
// get L7M_EINVAL, and the batcher is freed only after every caller inside
// l7m_batcher_eval* has read its verdict and left.
void l7m_batcher_destroy(l7m_batcher* b) {
  if (!b) return;
  {
    std::lock_guard<std::mutex> lk(b->mu);
    b->stop = true;
  }
  b->cv_flush.notify_all();
  for (auto& t : b->flushers)
    if (t.joinable()) t.join();
  {
    std::unique_lock<std::mutex> lk(b->mu);
    b->cv_idle.wait(lk, [&] { return b->callers.load() == 0; });
  }
  l7m_release(b->rs);
  for (Batch* x : b->all) delete x;
  delete b;
}

}  // extern "C"
