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
// a flusher thread evaluates the batch when it holds max_batch requests or
// its first request has waited max_delay_us, while the next batch fills.
// l7m_batcher_set_ruleset is the policy update (Redirect.updateRules,
// pkg/proxy/redirect.go:68-74): batches flushed afterwards use the new rules.
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/l7match.h"

namespace {

using Clock = std::chrono::steady_clock;

struct Batch {
  std::vector<uint8_t> arena;
  std::vector<uint64_t> offs;
  std::vector<uint32_t> ids;  // source identities (Kafka rule sets)
  std::vector<int32_t> verd;
  Clock::time_point first;
  bool done = false;
  int rc = L7M_OK;
};

}  // namespace

struct l7m_batcher {
  std::mutex mu;
  std::condition_variable cv_flush, cv_done;
  l7m_ruleset* rs = nullptr;
  uint32_t max_batch = 65536;
  uint32_t max_delay_us = 200;
  int device = 0;
  std::shared_ptr<Batch> cur = std::make_shared<Batch>();
  bool stop = false;
  uint64_t batches = 0, requests = 0;
  std::thread flusher;

  void run() {
    (void)hipSetDevice(device);
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      while (!stop && cur->offs.empty()) cv_flush.wait(lk);
      if (cur->offs.empty() && stop) return;
      // full, or the first request has waited long enough (or shutting down)
      const auto deadline = cur->first + std::chrono::microseconds(max_delay_us);
      while (!stop && cur->offs.size() < max_batch && Clock::now() < deadline) cv_flush.wait_until(lk, deadline);
      std::shared_ptr<Batch> b = cur;
      cur = std::make_shared<Batch>();
      l7m_ruleset* r = rs;
      l7m_retain(r);
      ++batches;
      requests += b->offs.size();
      lk.unlock();
      b->verd.resize(b->offs.size());
      b->arena.resize(b->arena.size() + 64, 0);  // tail padding for aligned loads
      l7m_ruleset_info info;
      l7m_ruleset_get_info(r, &info);
      const int rc = l7m_eval_ids(r, b->arena.data(), b->arena.size() - 64, b->offs.data(), b->offs.size(),
                                  info.proto == L7M_PROTO_KAFKA ? b->ids.data() : nullptr, b->verd.data(), nullptr,
                                  0);
      l7m_release(r);
      lk.lock();
      b->rc = rc;
      b->done = true;
      cv_done.notify_all();
    }
  }

  int eval(const uint8_t* rec, size_t len, uint32_t src_identity, int32_t* verdict) {
    std::unique_lock<std::mutex> lk(mu);
    if (stop) return L7M_EINVAL;
    std::shared_ptr<Batch> b = cur;
    const size_t idx = b->offs.size();
    if (idx == 0) b->first = Clock::now();
    const size_t off = b->arena.size();
    b->offs.push_back(off);
    b->ids.push_back(src_identity);
    b->arena.resize(off + ((len + 3) & ~size_t(3)), 0);
    if (len) std::memcpy(b->arena.data() + off, rec, len);
    if (idx == 0 || b->offs.size() >= max_batch) cv_flush.notify_one();
    cv_done.wait(lk, [&] { return b->done; });
    if (b->rc != L7M_OK) return b->rc;
    *verdict = b->verd[idx];
    return L7M_OK;
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
    b->device = o.device;
  }
  l7m_retain(rs);
  b->rs = rs;
  b->flusher = std::thread([b] { b->run(); });
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

void l7m_batcher_destroy(l7m_batcher* b) {
  if (!b) return;
  {
    std::lock_guard<std::mutex> lk(b->mu);
    b->stop = true;
  }
  b->cv_flush.notify_all();
  if (b->flusher.joinable()) b->flusher.join();
  l7m_release(b->rs);
  delete b;
}

}  // extern "C"
