// l7m_api.cc — the C ABI of libl7match.so (include/l7match.h).
//
// Compilation runs on the host (cold path); evaluation always runs on the GPU.
// There is no CPU evaluation path in this library: without a HIP device the
// eval entry points return L7M_EDEVICE.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/l7match.h"
#include "l7m_device.h"
#include "l7m_internal.h"
#include "program.h"

using namespace l7m;

namespace {

void set_err(char* err, size_t errlen, const std::string& m) {
  if (!err || errlen == 0) return;
  size_t k = m.size() < errlen - 1 ? m.size() : errlen - 1;
  std::memcpy(err, m.data(), k);
  err[k] = '\0';
}

// Older callers may pass a shorter l7m_opts (struct_size): copy what they set.
l7m_opts norm_opts(const l7m_opts* o) {
  l7m_opts r{};
  if (!o) return r;
  size_t k = o->struct_size == 0 || o->struct_size > sizeof(l7m_opts) ? sizeof(l7m_opts) : o->struct_size;
  std::memcpy(&r, o, k);
  return r;
}

int finish_compile(CompileResult&& cr, uint32_t proto, l7m_ruleset** out, char* err, size_t errlen) {
  if (cr.status != L7M_OK) {
    set_err(err, errlen, cr.err);
    return cr.status;
  }
  auto* rs = new (std::nothrow) l7m_ruleset();
  if (!rs) return L7M_ENOMEM;
  rs->proto = proto;
  rs->program = std::move(cr.program);
  rs->info = cr.info;
  rs->names = std::move(cr.names);
  rs->origin = std::move(cr.origin);
  *out = rs;
  return L7M_OK;
}

std::atomic<int> g_resident_cus[64];  // resident workgroups running per device (l7m_batch.cc)

int device_program(l7m_ruleset* rs, const uint32_t** out, int* cus) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return L7M_EDEVICE;
  if (dev < 0 || dev >= 64) return L7M_EDEVICE;
  hipDeviceProp_t prop;
  static thread_local int cached_dev = -1, cached_cus = 0;
  if (cached_dev != dev) {
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return L7M_EDEVICE;
    cached_dev = dev;
    cached_cus = prop.multiProcessorCount;
  }
  *cus = cached_cus;
  // fast path without the lock once the program is on this device (the
  // batcher's flushers launch concurrently on one rule set)
  if (void* q = __atomic_load_n(&rs->dprog[dev], __ATOMIC_ACQUIRE)) {
    *out = static_cast<const uint32_t*>(q);
    return L7M_OK;
  }
  std::lock_guard<std::mutex> g(rs->mu);
  if (!rs->dprog[dev]) {
    void* p = nullptr;
    size_t bytes = rs->program.size() * 4;
    if (hipMalloc(&p, bytes) != hipSuccess) return L7M_ENOMEM;
    if (hipMemcpy(p, rs->program.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(p);
      return L7M_EDEVICE;
    }
    __atomic_store_n(&rs->dprog[dev], p, __ATOMIC_RELEASE);
  }
  *out = static_cast<const uint32_t*>(rs->dprog[dev]);
  return L7M_OK;
}

// ---- Kafka compressed-message second pass: per-device scratch ------------
// The first pass queues the requests holding gzip / snappy messages;
// kafka_codec_kernel re-reads them with the values decoded in per-worker slabs.  Queues come from a small ring per device (a launch
// waits, on its stream, for the previous user of its queue); the slabs are
// one pool per device, so second passes of concurrent launches are chained
// through an event.  Without the scratch (allocation failure) the queue
// capacity is 0 and such requests report L7M_VERDICT_UNSUPPORTED.
constexpr int kCodecSlots = 8;
constexpr uint32_t kCodecQueueCap = 1u << 20;

struct KafkaCodecDev {
  std::mutex mu;
  bool init = false;
  uint8_t* slabs = nullptr;
  uint32_t workers = 0;
  uint64_t slab_bytes = 0;
  hipEvent_t p2_done = nullptr;
  struct Slot {
    uint32_t* recs = nullptr;
    uint32_t* qhdr = nullptr;
    uint32_t cap = 0;
    hipEvent_t done = nullptr;
    bool busy = false;  // claimed by a launch that has not recorded `done` yet
  } slots[kCodecSlots];
  uint32_t rr = 0;
  std::condition_variable cv;
};
KafkaCodecDev g_kcodec[64];

// Decode slabs are 2 x maxParseBufSize + 64 KiB (~13 MB) per worker, allocated
// at the first Kafka launch on a device: 16 workers ~ 211 MB.
uint32_t codec_workers() {
  const char* e = std::getenv("L7M_KAFKA_CODEC_WORKERS");
  const long v = e ? std::strtol(e, nullptr, 10) : 16;
  return v < 0 ? 0u : v > 4096 ? 4096u : static_cast<uint32_t>(v);
}

hipError_t launch_kafka_both(const uint32_t* dprog, const KafkaHeader& h, const uint8_t* arena, uint64_t arena_bytes,
                             const uint64_t* offs, uint64_t n, int32_t* verdicts, unsigned long long* hits,
                             hipStream_t stream, int cus, uint32_t flags, const uint32_t* ids) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  KafkaCodecDev& g = g_kcodec[dev];
  KafkaCodecQueue cq;
  KafkaCodecDev::Slot* slot = nullptr;
  {
    std::unique_lock<std::mutex> lk(g.mu);
    if (!g.init) {
      g.init = true;
      g.workers = codec_workers();
      // two decoded sets of maxParseBufSize always fit: nesting one level deep
      // never runs out of slab
      g.slab_bytes = (2ull * kKafkaMaxParseBuf + 65536 + 255) & ~255ull;
      if (g.workers && (hipMalloc(reinterpret_cast<void**>(&g.slabs), g.workers * g.slab_bytes) != hipSuccess ||
                        hipEventCreateWithFlags(&g.p2_done, hipEventDisableTiming) != hipSuccess)) {
        g.slabs = nullptr;
        g.workers = 0;
      }
    }
    for (;;) {  // a free queue: its previous user has enqueued its `done` record
      for (int k = 0; k < kCodecSlots && !slot; ++k) {
        KafkaCodecDev::Slot* c = &g.slots[g.rr++ % kCodecSlots];
        if (!c->busy) slot = c;
      }
      if (slot) break;
      g.cv.wait(lk);
    }
    slot->busy = true;
    if (!slot->qhdr || !slot->done) {  // first use, or a failed earlier initialisation: (re)try all of it
      if (slot->qhdr) (void)hipFree(slot->qhdr);
      if (slot->done) (void)hipEventDestroy(slot->done);
      slot->qhdr = nullptr;
      slot->done = nullptr;
      if (hipMalloc(reinterpret_cast<void**>(&slot->qhdr), 16) != hipSuccess || hipMemset(slot->qhdr, 0, 16) != hipSuccess ||
          hipEventCreateWithFlags(&slot->done, hipEventDisableTiming) != hipSuccess) {
        if (slot->qhdr) (void)hipFree(slot->qhdr);
        slot->qhdr = nullptr;
        slot->done = nullptr;
        slot->busy = false;
        g.cv.notify_one();
        return hipErrorOutOfMemory;
      }
    }
    if (g.workers && !slot->recs &&
        hipMalloc(reinterpret_cast<void**>(&slot->recs), kCodecQueueCap * sizeof(uint32_t)) == hipSuccess)
      slot->cap = kCodecQueueCap;  // retried on later launches when it failed
    // the queue header is zero here: reset by the previous user's second
    // pass (kafka_codec_kernel) or by the memset after a launch without one
    hipError_t e = hipStreamWaitEvent(stream, slot->done, 0);
    if (e != hipSuccess) {
      slot->busy = false;
      return e;
    }
    cq.recs = slot->recs;
    cq.qhdr = slot->qhdr;
    cq.cap = g.workers ? slot->cap : 0;
    cq.workers = g.workers;
    cq.slabs = g.slabs;
    cq.slab_bytes = g.slab_bytes;
  }
  hipError_t e = launch_kafka(dprog, h, arena, arena_bytes, offs, n, verdicts, hits, stream, cus, flags, cq, ids);
  std::lock_guard<std::mutex> lk(g.mu);
  if (e == hipSuccess && n && !(flags & (L7M_FLAG_DIAG_COPY_ONLY | L7M_FLAG_DIAG_WALK_ONLY)) && cq.cap &&
      cq.workers) {
    e = hipStreamWaitEvent(stream, g.p2_done, 0);
    if (e == hipSuccess) e = launch_kafka_codec(dprog, arena, arena_bytes, offs, n, verdicts, hits, stream, cq);
    if (e == hipSuccess) e = hipEventRecord(g.p2_done, stream);
  } else if (e == hipSuccess && n) {
    e = hipMemsetAsync(slot->qhdr, 0, 16, stream);  // no second pass to reset the queue header
  }
  const hipError_t e2 = hipEventRecord(slot->done, stream);
  if (e == hipSuccess) e = e2;
  slot->busy = false;
  g.cv.notify_one();
  return e;
}

int launch(const l7m_ruleset* crs, const void* arena, size_t arena_bytes, const void* offs, size_t n, void* verdicts,
           void* hits, hipStream_t stream, uint32_t flags, const void* ids = nullptr,
           const DoneSignal* done = nullptr, bool* signalled = nullptr) {
  if (signalled) *signalled = false;
  auto* rs = const_cast<l7m_ruleset*>(crs);
  const uint32_t* dprog = nullptr;
  int cus = 0;
  int rc = device_program(rs, &dprog, &cus);
  if (rc != L7M_OK) return rc;
  {
    // resident batcher workgroups each hold a CU: a persistent grid sized to
    // every CU would leave its last workgroup waiting for another to finish
    int dev = 0;
    (void)hipGetDevice(&dev);
    const int busy = dev >= 0 && dev < 64 ? g_resident_cus[dev].load(std::memory_order_relaxed) : 0;
    if (busy > 0) cus = cus - busy > 1 ? cus - busy : 1;
  }
  hipError_t e;
  if (rs->proto == L7M_PROTO_HTTP) {
    if (ids) return L7M_EINVAL;  // HTTP records carry their remote identity
    HttpHeader h;
    std::memcpy(&h, rs->program.data(), sizeof h);
    if (http_stage_bytes(h) == 0) return L7M_ETOOBIG;
    const DfaDesc* dd = reinterpret_cast<const DfaDesc*>(rs->program.data() + h.off_dfas);
    for (uint32_t k = 0; k < h.n_dfas; ++k)
      if (dd[k].lit_tab != kNone) flags |= kLaunchLiterals;
    e = launch_http(dprog, h, static_cast<const uint8_t*>(arena), arena_bytes, static_cast<const uint64_t*>(offs),
                    n, static_cast<int32_t*>(verdicts), static_cast<unsigned long long*>(hits),
                    stream, cus, flags, done);
    if (signalled) *signalled = done && n && !h.n_slow && e == hipSuccess;
  } else if (rs->proto == L7M_PROTO_KAFKA) {
    KafkaHeader h;
    std::memcpy(&h, rs->program.data(), sizeof h);
    e = launch_kafka_both(dprog, h, static_cast<const uint8_t*>(arena), arena_bytes,
                          static_cast<const uint64_t*>(offs), n, static_cast<int32_t*>(verdicts),
                          static_cast<unsigned long long*>(hits), stream, cus, flags,
                          static_cast<const uint32_t*>(ids));
  } else {
    return L7M_EINVAL;
  }
  return e == hipSuccess ? L7M_OK : L7M_EDEVICE;
}


// ---- l7m_eval contexts ------------------------------------------------------
// l7m_eval is reentrant: each concurrent call takes its own context (stream +
// device buffers grown to the largest batch seen) from a per-device free
// list, so steady-state calls allocate nothing and never share buffers.
constexpr int kMaxDevices = 64;

struct EvalCtx {
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // second stream of the chunked pipeline (lazily created)
  hipEvent_t ev = nullptr, ev2 = nullptr;
  void *arena = nullptr, *offs = nullptr, *verd = nullptr, *hits = nullptr, *ids = nullptr;
  size_t cap_arena = 0, cap_offs = 0, cap_verd = 0, cap_hits = 0, cap_ids = 0;
  std::vector<uint64_t> hhost;
  static int grow(void** p, size_t* cap, size_t want) {
    if (*cap >= want) return L7M_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t sz = want + want / 4;  // some headroom for the next batch
    if (hipMalloc(p, sz) != hipSuccess) {
      *p = nullptr;
      return L7M_ENOMEM;
    }
    *cap = sz;
    return L7M_OK;
  }
  int reserve(size_t abytes, size_t n, size_t nctr, bool with_ids) {
    int rc = grow(&arena, &cap_arena, abytes);
    if (rc == L7M_OK && with_ids) rc = grow(&ids, &cap_ids, n * 4);
    if (rc == L7M_OK) rc = grow(&offs, &cap_offs, n * 8);
    if (rc == L7M_OK) rc = grow(&verd, &cap_verd, n * 4);
    if (rc == L7M_OK) rc = grow(&hits, &cap_hits, nctr * 8);
    if (rc == L7M_OK) hhost.resize(nctr);
    return rc;
  }
};

struct CtxPool {
  std::mutex mu;
  std::vector<EvalCtx*> free;
};
CtxPool g_pools[kMaxDevices];

EvalCtx* acquire_ctx(int dev) {
  {
    std::lock_guard<std::mutex> g(g_pools[dev].mu);
    if (!g_pools[dev].free.empty()) {
      EvalCtx* c = g_pools[dev].free.back();
      g_pools[dev].free.pop_back();
      return c;
    }
  }
  auto* c = new (std::nothrow) EvalCtx();
  if (!c) return nullptr;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return nullptr;
  }
  return c;
}

void release_ctx(int dev, EvalCtx* c) {
  std::lock_guard<std::mutex> g(g_pools[dev].mu);
  g_pools[dev].free.push_back(c);
}

// Large host batches are pipelined: the arena is cut at record boundaries
// into chunks of ~kPipeChunkBytes, and chunk k's H2D copy, kernel and D2H of
// verdicts are enqueued on stream k & 1, so chunk k+1's copy overlaps chunk
// k's kernel (SURVEY.md §8(d) end-to-end).  The device arena keeps the host
// layout (offsets stay valid); the kernels read only their own chunk's
// records.  Needs ascending offsets (what every packer produces); other
// batches take the one-shot path.  Pass pinned memory (l7m_alloc_pinned) for
// DMA-rate copies.
constexpr size_t kPipeChunkBytes = size_t(64) << 20;

bool ascending(const uint64_t* offs, size_t n, size_t arena_bytes) {
  for (size_t i = 1; i < n; ++i)
    if (offs[i] < offs[i - 1]) return false;
  return n == 0 || offs[n - 1] < arena_bytes;
}

// Zero-copy: a host buffer the device can address (pinned by hipHostMalloc /
// l7m_alloc_pinned, mapped into the device's address space) is read by the
// kernels in place over PCIe instead of being copied first (config 2, 2 GB:
// 54.7 GB/s against 36.5 GB/s for the chunked H2D pipeline,
// tools/zero_copy_probe.py).  Returns the device address of [p, p + bytes)
// only when the runtime reports that whole range inside ONE device-mapped
// host allocation, else nullptr (the caller copies).  L7M_ZERO_COPY=0
// disables it.
const void* mapped_host_range(const void* p, size_t bytes) {
  static const bool enabled = [] {
    const char* e = std::getenv("L7M_ZERO_COPY");
    return !(e && e[0] == '0');
  }();
  if (!enabled || !p || !bytes) return nullptr;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: not an error here
    return nullptr;
  }
  if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, a.devicePointer) != hipSuccess || !base) {
    (void)hipGetLastError();
    return nullptr;
  }
  const auto d = reinterpret_cast<uintptr_t>(a.devicePointer), b = reinterpret_cast<uintptr_t>(base);
  if (d < b || d - b > size || bytes > size - (d - b)) return nullptr;
  return a.devicePointer;
}

int eval_pipelined(EvalCtx* c, const l7m_ruleset* rs, const uint8_t* arena, size_t arena_bytes,
                   const uint64_t* offsets, size_t n, const uint32_t* ids, int32_t* verdicts, bool hits,
                   size_t abytes, size_t nctr, uint32_t flags) {
  if (!c->stream2 && hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess) return L7M_EDEVICE;
  if (!c->ev && hipEventCreateWithFlags(&c->ev, hipEventDisableTiming) != hipSuccess) return L7M_EDEVICE;
  if (!c->ev2 && hipEventCreateWithFlags(&c->ev2, hipEventDisableTiming) != hipSuccess) return L7M_EDEVICE;
  const hipStream_t s0 = c->stream, s1 = c->stream2;
  auto* da = static_cast<uint8_t*>(c->arena);
  auto* doffs = static_cast<uint64_t*>(c->offs);
  auto* dverd = static_cast<int32_t*>(c->verd);
  auto* dids = static_cast<uint32_t*>(c->ids);
  bool ok = hipMemsetAsync(da + arena_bytes, 0, abytes - arena_bytes, s0) == hipSuccess &&
            (!hits || hipMemsetAsync(c->hits, 0, nctr * 8, s0) == hipSuccess) &&
            hipEventRecord(c->ev, s0) == hipSuccess && hipStreamWaitEvent(s1, c->ev, 0) == hipSuccess;
  int rc = ok ? L7M_OK : L7M_EDEVICE;
  size_t lo = 0;
  for (int k = 0; rc == L7M_OK && lo < n; ++k) {
    const uint64_t a = k == 0 ? 0 : offsets[lo];
    // first record starting at or past a + chunk: the chunk ends there
    size_t hi = static_cast<size_t>(std::lower_bound(offsets + lo, offsets + n, a + kPipeChunkBytes) - offsets);
    if (hi == lo) hi = lo + 1;
    const uint64_t b = hi < n ? offsets[hi] : arena_bytes;
    const hipStream_t st = (k & 1) ? s1 : s0;
    ok = hipMemcpyAsync(da + a, arena + a, b - a, hipMemcpyHostToDevice, st) == hipSuccess &&
         hipMemcpyAsync(doffs + lo, offsets + lo, (hi - lo) * 8, hipMemcpyHostToDevice, st) == hipSuccess &&
         (!ids || hipMemcpyAsync(dids + lo, ids + lo, (hi - lo) * 4, hipMemcpyHostToDevice, st) == hipSuccess);
    if (!ok) rc = L7M_EDEVICE;
    if (rc == L7M_OK)
      rc = launch(rs, da, arena_bytes, doffs + lo, hi - lo, dverd + lo, hits ? c->hits : nullptr, st, flags,
                  ids ? dids + lo : nullptr);
    if (rc == L7M_OK &&
        hipMemcpyAsync(verdicts + lo, dverd + lo, (hi - lo) * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
      rc = L7M_EDEVICE;
    lo = hi;
  }
  // join: stream 0 waits for stream 1, then the counters come back
  if (hipEventRecord(c->ev2, s1) != hipSuccess || hipStreamWaitEvent(s0, c->ev2, 0) != hipSuccess) rc = L7M_EDEVICE;
  if (rc == L7M_OK && hits &&
      hipMemcpyAsync(c->hhost.data(), c->hits, nctr * 8, hipMemcpyDeviceToHost, s0) != hipSuccess)
    rc = L7M_EDEVICE;
  if (hipStreamSynchronize(s0) != hipSuccess && rc == L7M_OK) rc = L7M_EDEVICE;
  if (hipStreamSynchronize(s1) != hipSuccess && rc == L7M_OK) rc = L7M_EDEVICE;
  return rc;
}

}  // namespace

namespace l7m {

// The batcher's resident evaluator (l7m_batch.cc): whether the rule set can
// be served by kafka_resident_kernel, with its device program, instantiation,
// record stage and serial.
void resident_running(int dev, int delta) {
  if (dev >= 0 && dev < 64) g_resident_cus[dev].fetch_add(delta, std::memory_order_relaxed);
}

bool resident_program(l7m_ruleset* rs, const uint32_t** dprog, int* kind, uint32_t* stage, uint64_t* serial) {
  // Kafka only: for HTTP the launch per batch measured faster (config 2, 8
  // callers: 165 k/s at p50 47 us launched vs 158 k/s at p50 51 us resident,
  // profiles/r04/ab_round4.md)
  if (rs->proto != L7M_PROTO_KAFKA) return false;
  int cus = 0;
  if (device_program(rs, dprog, &cus) != L7M_OK) return false;
  *serial = rs->serial;
  KafkaHeader kh;
  std::memcpy(&kh, rs->program.data(), sizeof kh);
  return kafka_resident_ok(kh, kind, stage);
}

// The batcher's latency path (l7m_batch.cc): l7m_eval_device on device-visible
// buffers with the kernel's completion signal (l7m_device.h DoneSignal) when
// one launch decides every request (HTTP without a slow pass); *signalled
// false means the caller waits on the stream instead.
int eval_device_signal(const l7m_ruleset* rs, const void* d_arena, size_t arena_bytes, const void* d_offs, size_t n,
                       void* d_verdicts, hipStream_t stream, const DoneSignal& sig, bool* signalled) {
  *signalled = false;
  if (!rs || (n && (!d_arena || !d_offs || !d_verdicts))) return L7M_EINVAL;
  if (reinterpret_cast<uintptr_t>(d_arena) & 15) return L7M_EINVAL;
  if (rs->proto != L7M_PROTO_HTTP) return launch(rs, d_arena, arena_bytes, d_offs, n, d_verdicts, nullptr, stream, 0);
  return launch(rs, d_arena, arena_bytes, d_offs, n, d_verdicts, nullptr, stream, 0, nullptr, &sig, signalled);
}

}  // namespace l7m

extern "C" {

int l7m_abi_version(void) { return L7M_ABI_VERSION; }

int l7m_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int l7m_compile_http(const l7m_http_rule* rules, size_t n, const l7m_opts* opts, l7m_ruleset** out,
                     char* err, size_t errlen) {
  if (!out) return L7M_EINVAL;
  try {
    return finish_compile(compile_http(rules, n, norm_opts(opts)), L7M_PROTO_HTTP, out, err, errlen);
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "out of host memory");
    return L7M_ENOMEM;
  }
}

int l7m_compile_kafka(const l7m_kafka_rule* rules, size_t n, const l7m_opts* opts,
                      l7m_ruleset** out, char* err, size_t errlen) {
  if (!out) return L7M_EINVAL;
  try {
    return finish_compile(compile_kafka(rules, n, norm_opts(opts)), L7M_PROTO_KAFKA, out, err, errlen);
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "out of host memory");
    return L7M_ENOMEM;
  }
}

int l7m_compile_kafka_map(const l7m_kafka_selector_rules* map, size_t n_entries,
                          const l7m_identity_selectors* identities, size_t n_identities, const l7m_opts* opts,
                          l7m_ruleset** out, char* err, size_t errlen) {
  if (!out) return L7M_EINVAL;
  try {
    return finish_compile(compile_kafka_map(map, n_entries, identities, n_identities, norm_opts(opts)),
                          L7M_PROTO_KAFKA, out, err, errlen);
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "out of host memory");
    return L7M_ENOMEM;
  }
}

int l7m_compile_http_policies(const l7m_network_policy* policies, size_t n, const l7m_opts* opts,
                              l7m_ruleset** out, char* err, size_t errlen) {
  if (!out) return L7M_EINVAL;
  try {
    return finish_compile(compile_http_policies(policies, n, norm_opts(opts)), L7M_PROTO_HTTP, out, err, errlen);
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "out of host memory");
    return L7M_ENOMEM;
  }
}

int l7m_ruleset_policy_index(const l7m_ruleset* rs, const char* name) {
  if (!rs || !name || rs->proto != L7M_PROTO_HTTP) return -1;
  for (size_t i = 0; i < rs->names.size(); ++i)
    if (rs->names[i] == name) return static_cast<int>(i);
  return -1;
}

int l7m_ruleset_rule_origin(const l7m_ruleset* rs, uint32_t rule, l7m_rule_origin* out) {
  if (!rs || !out || rs->proto != L7M_PROTO_HTTP || rule >= rs->origin.size()) return L7M_EINVAL;
  *out = rs->origin[rule];
  return L7M_OK;
}

void l7m_retain(l7m_ruleset* rs) {
  if (rs) rs->refs.fetch_add(1);
}

void l7m_release(l7m_ruleset* rs) {
  if (!rs) return;
  if (rs->refs.fetch_sub(1) != 1) return;
  for (int d = 0; d < 64; ++d)
    if (rs->dprog[d]) {
      int cur = 0;
      (void)hipGetDevice(&cur);
      (void)hipSetDevice(d);
      (void)hipFree(rs->dprog[d]);
      (void)hipSetDevice(cur);
    }
  delete rs;
}

int l7m_ruleset_get_info(const l7m_ruleset* rs, l7m_ruleset_info* out) {
  if (!rs || !out) return L7M_EINVAL;
  *out = rs->info;
  return L7M_OK;
}

int l7m_ruleset_program(const l7m_ruleset* rs, void* buf, size_t* len) {
  if (!rs || !len) return L7M_EINVAL;
  size_t bytes = rs->program.size() * 4;
  if (buf) {
    if (*len < bytes) return L7M_EINVAL;
    std::memcpy(buf, rs->program.data(), bytes);
  }
  *len = bytes;
  return L7M_OK;
}

int l7m_http_translate(const l7m_http_rule* rule, l7m_header_matcher* out, size_t cap, char* err,
                       size_t errlen) {
  if (!rule) return L7M_EINVAL;
  static thread_local std::vector<HeaderMatcher> hm;
  std::string e;
  int rc = translate_http_rule(*rule, &hm, &e);
  if (rc != L7M_OK) {
    set_err(err, errlen, e);
    return rc;
  }
  for (size_t i = 0; i < hm.size() && i < cap && out; ++i) {
    out[i].name = hm[i].name.c_str();
    out[i].value = hm[i].value.c_str();
    out[i].kind = static_cast<uint32_t>(envoy_kind(hm[i]));
    out[i].has_regex_flag = hm[i].has_regex ? 1u : 0u;
  }
  return static_cast<int>(hm.size());
}

size_t l7m_http_record_size(const l7m_http_request* q) {
  if (!q) return 0;
  auto len = [](const char* s) -> size_t { return s ? std::strlen(s) : 0; };
  size_t ml = len(q->method), pl = len(q->path), al = len(q->authority);
  if (ml > 0xffff || pl > 0xffff || al > 0xffff || q->n_headers > 255) return 0;
  size_t b = L7M_HTTP_REC_FIXED + 4u * q->n_headers + ml + pl + al;
  for (uint32_t j = 0; j < q->n_headers; ++j) {
    size_t nl = len(q->header_names[j]), vl = len(q->header_values[j]);
    if (nl > 0xffff || vl > 0xffff) return 0;
    b += nl + vl;
  }
  if (b > 0xffffffffu) return 0;
  return (b + 3) & ~size_t(3);
}

size_t l7m_pack_http(const l7m_http_request* reqs, size_t n, uint8_t* arena, size_t cap,
                     uint64_t* offsets) {
  size_t used = 0;
  for (size_t i = 0; i < n; ++i) {
    const l7m_http_request& q = reqs[i];
    size_t sz = l7m_http_record_size(&q);
    if (sz == 0 || used + sz > cap) return 0;
    uint8_t* r = arena + used;
    std::memset(r, 0, sz);
    auto len = [](const char* s) -> uint32_t { return s ? static_cast<uint32_t>(std::strlen(s)) : 0; };
    uint32_t ml = len(q.method), pl = len(q.path), al = len(q.authority);
    uint32_t flags = (q.method ? L7M_HTTP_F_METHOD : 0) | (q.path ? L7M_HTTP_F_PATH : 0) |
                     (q.authority ? L7M_HTTP_F_AUTHORITY : 0) | (q.ingress ? L7M_HTTP_F_INGRESS : 0);
    uint32_t w[5];
    size_t unpadded = L7M_HTTP_REC_FIXED + 4u * q.n_headers + ml + pl + al;
    for (uint32_t j = 0; j < q.n_headers; ++j) unpadded += len(q.header_names[j]) + len(q.header_values[j]);
    w[0] = static_cast<uint32_t>(unpadded);
    w[1] = q.remote_id;
    w[2] = q.dport | (flags << 16) | (q.n_headers << 24);
    w[3] = ml | (pl << 16);
    w[4] = al | (std::min<uint32_t>(q.policy, L7M_POLICY_UNKNOWN) << 16);
    std::memcpy(r, w, sizeof w);
    size_t p = L7M_HTTP_REC_FIXED;
    for (uint32_t j = 0; j < q.n_headers; ++j) {
      uint32_t e = len(q.header_names[j]) | (len(q.header_values[j]) << 16);
      std::memcpy(r + p, &e, 4);
      p += 4;
    }
    auto put = [&](const char* s, uint32_t l) {
      if (l) std::memcpy(r + p, s, l);
      p += l;
    };
    put(q.method, ml);
    put(q.path, pl);
    put(q.authority, al);
    for (uint32_t j = 0; j < q.n_headers; ++j) {
      uint32_t nl = len(q.header_names[j]);
      for (uint32_t k = 0; k < nl; ++k) {
        char c = q.header_names[j][k];
        r[p + k] = static_cast<uint8_t>((c >= 'A' && c <= 'Z') ? c - 'A' + 'a' : c);
      }
      p += nl;
      put(q.header_values[j], len(q.header_values[j]));
    }
    offsets[i] = used;
    used += sz;
  }
  return used;
}

int l7m_eval_device(const l7m_ruleset* rs, const void* d_arena, size_t arena_bytes,
                    const void* d_offsets, size_t n, void* d_verdicts, void* d_hits,
                    void* hip_stream, uint32_t flags) {
  if (!rs || (n && (!d_arena || !d_offsets || !d_verdicts))) return L7M_EINVAL;
  // The kernels stream records with aligned 16-byte loads.
  if (reinterpret_cast<uintptr_t>(d_arena) & 15) return L7M_EINVAL;
  return launch(rs, d_arena, arena_bytes, d_offsets, n, d_verdicts, d_hits, static_cast<hipStream_t>(hip_stream),
                flags);
}

int l7m_eval_device_ids(const l7m_ruleset* rs, const void* d_arena, size_t arena_bytes, const void* d_offsets,
                        size_t n, const void* d_ids, void* d_verdicts, void* d_hits, void* hip_stream,
                        uint32_t flags) {
  if (!rs || (n && (!d_arena || !d_offsets || !d_verdicts))) return L7M_EINVAL;
  if (reinterpret_cast<uintptr_t>(d_arena) & 15) return L7M_EINVAL;
  if (rs->proto != L7M_PROTO_KAFKA) return L7M_EINVAL;
  return launch(rs, d_arena, arena_bytes, d_offsets, n, d_verdicts, d_hits, static_cast<hipStream_t>(hip_stream),
                flags, d_ids);
}

int l7m_eval(const l7m_ruleset* rs, const uint8_t* arena, size_t arena_bytes,
             const uint64_t* offsets, size_t n, int32_t* verdicts, uint64_t* hits, uint32_t flags) {
  return l7m_eval_ids(rs, arena, arena_bytes, offsets, n, nullptr, verdicts, hits, flags);
}

int l7m_eval_ids(const l7m_ruleset* rs, const uint8_t* arena, size_t arena_bytes, const uint64_t* offsets,
                 size_t n, const uint32_t* ids, int32_t* verdicts, uint64_t* hits, uint32_t flags) {
  if (!rs || (n && (!arena || !offsets || !verdicts))) return L7M_EINVAL;
  if (ids && rs->proto != L7M_PROTO_KAFKA) return L7M_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return L7M_EDEVICE;
  if (n == 0) return L7M_OK;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return L7M_EDEVICE;
  const size_t nctr = rs->info.n_counters;
  // Pad the arena copy so that the kernels' aligned word loads never run past it.
  const size_t abytes = (arena_bytes + 64) & ~size_t(3);
  EvalCtx* c = acquire_ctx(dev);
  if (!c) return L7M_EDEVICE;
  // zero-copy when the padded arena is device-mapped host memory (the
  // kernels' aligned over-reads stay inside [arena, arena + abytes))
  const void* za = (reinterpret_cast<uintptr_t>(arena) & 15) ? nullptr : mapped_host_range(arena, abytes);
  int rc = c->reserve(za ? 0 : abytes, n, nctr, ids != nullptr);
  if (rc == L7M_OK && za) {
    const hipStream_t st = c->stream;
    const void* zo = (reinterpret_cast<uintptr_t>(offsets) & 7) ? nullptr : mapped_host_range(offsets, n * 8);
    const void* zi = ids && !(reinterpret_cast<uintptr_t>(ids) & 3) ? mapped_host_range(ids, n * 4) : nullptr;
    bool ok = (zo || hipMemcpyAsync(c->offs, offsets, n * 8, hipMemcpyHostToDevice, st) == hipSuccess) &&
              (!ids || zi || hipMemcpyAsync(c->ids, ids, n * 4, hipMemcpyHostToDevice, st) == hipSuccess) &&
              (!hits || hipMemsetAsync(c->hits, 0, nctr * 8, st) == hipSuccess);
    if (!ok) rc = L7M_EDEVICE;
    if (rc == L7M_OK)
      rc = launch(rs, za, arena_bytes, zo ? zo : c->offs, n, c->verd, hits ? c->hits : nullptr, st, flags,
                  ids ? (zi ? zi : c->ids) : nullptr);
    if (rc == L7M_OK && hipMemcpyAsync(verdicts, c->verd, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
      rc = L7M_EDEVICE;
    if (rc == L7M_OK && hits && hipMemcpyAsync(c->hhost.data(), c->hits, nctr * 8, hipMemcpyDeviceToHost, st) != hipSuccess)
      rc = L7M_EDEVICE;
    if (hipStreamSynchronize(st) != hipSuccess && rc == L7M_OK) rc = L7M_EDEVICE;
    if (rc == L7M_OK && hits)
      for (size_t i = 0; i < nctr; ++i) hits[i] += c->hhost[i];
  } else if (rc == L7M_OK && arena_bytes >= 2 * kPipeChunkBytes && ascending(offsets, n, arena_bytes)) {
    rc = eval_pipelined(c, rs, arena, arena_bytes, offsets, n, ids, verdicts, hits != nullptr, abytes, nctr, flags);
    if (rc == L7M_OK && hits)
      for (size_t i = 0; i < nctr; ++i) hits[i] += c->hhost[i];
  } else if (rc == L7M_OK) {
    const hipStream_t st = c->stream;
    bool ok = hipMemsetAsync(static_cast<uint8_t*>(c->arena) + arena_bytes, 0, abytes - arena_bytes, st) == hipSuccess &&
              hipMemcpyAsync(c->arena, arena, arena_bytes, hipMemcpyHostToDevice, st) == hipSuccess &&
              hipMemcpyAsync(c->offs, offsets, n * 8, hipMemcpyHostToDevice, st) == hipSuccess &&
              (!ids || hipMemcpyAsync(c->ids, ids, n * 4, hipMemcpyHostToDevice, st) == hipSuccess) &&
              (!hits || hipMemsetAsync(c->hits, 0, nctr * 8, st) == hipSuccess);
    if (!ok) rc = L7M_EDEVICE;
    if (rc == L7M_OK)
      rc = launch(rs, c->arena, arena_bytes, c->offs, n, c->verd, hits ? c->hits : nullptr, st, flags,
                  ids ? c->ids : nullptr);
    if (rc == L7M_OK && hipMemcpyAsync(verdicts, c->verd, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
      rc = L7M_EDEVICE;
    if (rc == L7M_OK && hits && hipMemcpyAsync(c->hhost.data(), c->hits, nctr * 8, hipMemcpyDeviceToHost, st) != hipSuccess)
      rc = L7M_EDEVICE;
    if (hipStreamSynchronize(st) != hipSuccess && rc == L7M_OK) rc = L7M_EDEVICE;
    if (rc == L7M_OK && hits)
      for (size_t i = 0; i < nctr; ++i) hits[i] += c->hhost[i];
  }
  release_ctx(dev, c);
  return rc;
}

int l7m_alloc_pinned(size_t bytes, void** out) {
  if (!out) return L7M_EINVAL;
  return hipHostMalloc(out, bytes, hipHostMallocDefault) == hipSuccess ? L7M_OK : L7M_ENOMEM;
}

void l7m_free_pinned(void* p) {
  if (p) (void)hipHostFree(p);
}

int l7m_host_mapped(const void* p, size_t bytes) { return mapped_host_range(p, bytes) ? 1 : 0; }

}  // extern "C"
