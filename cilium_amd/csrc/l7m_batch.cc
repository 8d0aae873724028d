// l7m_batch.cc — the batching front-end of the verdict path (l7m_batcher in
// include/l7match.h).
//
// The reference decides one request per call on the connection's own
// goroutine / Envoy worker: canAccess -> MatchesRule (pkg/proxy/kafka.go:116-152,
// called from handleRequest :232-306) and AccessFilter::decodeHeaders ->
// NetworkPolicyMap::Allowed (envoy/cilium_l7policy.cc:126-186).  A GPU call
// per request would cost more than the verdict, so the batcher keeps that
// per-request, blocking call shape while many callers' requests share one
// evaluation: a caller appends its record to the batch being filled and
// waits; a flusher evaluates the batch (eagerly, as soon as it is free, or
// when max_batch are pending / the first has waited max_delay_us) while the
// next batch fills.
//
// Latency path (round 4):
//   * append without a lock: a caller reserves its slot and its arena bytes
//     with one compare-and-swap on the batch's reservation word (count,
//     bytes, closed bit), copies its record and bumps `written`;
//   * batches are preallocated pinned, device-mapped host buffers (arena,
//     offsets, identities, verdicts): the kernels read the records and write
//     the verdicts in place over PCIe (l7m_eval_device on the mapped
//     pointers), no staging copies;
//   * a flusher closes the batch (sets the closed bit, installs a fresh
//     batch), waits for the reserved slots to be written, enqueues the
//     kernels on its own stream and polls for completion: HTTP launches
//     store a sequence number to a pinned host word once every verdict is
//     visible (round 6, l7m_device.h DoneSignal), other launches are
//     followed by an event;
//   * callers spin briefly on the batch's done flag, then sleep on its
//     condition variable.
// l7m_batcher_get_profile breaks the per-batch time into these phases.
// l7m_batcher_set_ruleset is the policy update (Redirect.updateRules,
// pkg/proxy/redirect.go:68-74): batches flushed afterwards use the new rules.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/l7match.h"
#include "l7m_device.h"

namespace l7m {
bool resident_program(l7m_ruleset* rs, const uint32_t** dprog, int* kind, uint32_t* stage, uint64_t* serial);
int eval_device_signal(const l7m_ruleset* rs, const void* d_arena, size_t arena_bytes, const void* d_offs, size_t n,
                       void* d_verdicts, hipStream_t stream, const DoneSignal& sig, bool* signalled);
void resident_running(int dev, int delta);  // persistent grids leave those CUs out (l7m_api.cc)
}

namespace {

using Clock = std::chrono::steady_clock;
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}
inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}

// Reservation word of a batch: closed bit | record count << 40 | arena bytes.
constexpr uint64_t kClosed = 1ull << 63;
constexpr int kCountShift = 40;
constexpr uint64_t kBytesMask = (1ull << kCountShift) - 1;
constexpr uint32_t count_of(uint64_t s) { return static_cast<uint32_t>((s & ~kClosed) >> kCountShift); }
constexpr uint64_t bytes_of(uint64_t s) { return s & kBytesMask; }
constexpr int64_t kSpinNs = 50000;  // a caller spins this long for its verdict, then sleeps

struct Batch {
  // one pinned, device-mapped allocation: arena (arena_cap + 64 bytes of
  // readable slack) | offsets | identities | verdicts
  void* host = nullptr;
  uint8_t* arena = nullptr;
  uint64_t* offs = nullptr;
  uint32_t* ids = nullptr;
  int32_t* verd = nullptr;
  const void *d_arena = nullptr, *d_offs = nullptr, *d_ids = nullptr;
  void* d_verd = nullptr;
  size_t arena_cap = 0;
  uint32_t cap = 0;
  std::atomic<uint64_t> resv{0};
  std::atomic<uint32_t> written{0};  // reserved slots whose record is in place
  std::atomic<uint32_t> done{0};
  std::atomic<uint32_t> readers{0};  // callers that have not read their verdict yet
  std::atomic<uint32_t> sleepers{0};
  std::atomic<uint32_t> want_close{0};  // a caller found no room
  std::atomic<int64_t> first_ns{0};
  int64_t done_ns = 0;
  int rc = L7M_OK;
  std::mutex m;
  std::condition_variable cv;

  bool alloc(size_t acap, uint32_t rcap) {
    const size_t a = (acap + 64 + 255) & ~size_t(255);
    const size_t o = (static_cast<size_t>(rcap) * 8 + 255) & ~size_t(255);
    const size_t i = (static_cast<size_t>(rcap) * 4 + 255) & ~size_t(255);
    const size_t v = static_cast<size_t>(rcap) * 4;
    if (hipHostMalloc(&host, a + o + i + v, hipHostMallocMapped) != hipSuccess) {
      host = nullptr;
      return false;
    }
    uint8_t* p = static_cast<uint8_t*>(host);
    arena = p;
    offs = reinterpret_cast<uint64_t*>(p + a);
    ids = reinterpret_cast<uint32_t*>(p + a + o);
    verd = reinterpret_cast<int32_t*>(p + a + o + i);
    std::memset(arena, 0, a);
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess || !d) return false;
    uint8_t* dp = static_cast<uint8_t*>(d);
    d_arena = dp;
    d_offs = dp + a;
    d_ids = dp + a + o;
    d_verd = dp + a + o + i;
    arena_cap = acap;
    cap = rcap;
    return true;
  }
  ~Batch() {
    if (host) (void)hipHostFree(host);
  }
  // A caller holding a stale `cur` snapshot may CAS a slot into this batch as
  // soon as resv loses its closed bit, so every other field is cleared first
  // and resv last (release): such a caller then sees done == 0, readers == 0.
  void reset() {
    written.store(0);
    done.store(0);
    readers.store(0);
    sleepers.store(0);
    want_close.store(0);
    first_ns.store(0);
    rc = L7M_OK;
    resv.store(0, std::memory_order_release);
  }
};

}  // namespace

struct l7m_batcher {
  uint32_t max_batch = 65536;
  uint32_t max_delay_us = 200;
  uint32_t in_flight = 4;
  bool eager = false;
  int device = 0;
  size_t arena_cap = 16u << 20;
  std::atomic<Batch*> cur{nullptr};
  std::mutex rs_mu;  // guards rs
  l7m_ruleset* rs = nullptr;
  std::mutex close_mu;  // flushers: close a batch + install the next
  std::mutex pool_mu;   // guards pool, all
  std::vector<Batch*> pool, all;
  std::atomic<bool> stop{false};
  std::atomic<uint32_t> callers{0};
  std::atomic<uint32_t> in_closed{0};  // callers waiting on a batch that is already being evaluated
  std::atomic<uint32_t> idle{0};  // flushers asleep
  std::mutex idle_mu;
  std::condition_variable idle_cv;
  std::vector<std::thread> flushers;
  // statistics (l7m_batcher_stats / l7m_batcher_get_profile)
  std::atomic<uint64_t> batches{0}, requests{0}, fill_ns{0}, fill_batches{0}, launch_ns{0}, gpu_ns{0}, wake_ns{0};
  std::atomic<uint64_t> res_batches{0}, res_read{0}, res_eval{0}, res_sync{0};  // device ticks (100 MHz)

  // Resident evaluator (l7m_kafka.hip kafka_resident_kernel): Kafka batches
  // of up to kResidentMax records are posted to a workgroup that stays on the
  // GPU instead of launching the first pass and the codec pass each (config
  // 3, 8 callers: 105 k/s at p50 72 us launched -> 163-177 k/s at p50 45-49
  // us).  HTTP batches are launched: the resident HTTP workgroup measured
  // slower than a launch (profiles/r04/ab_round4.md).
  static constexpr uint32_t kResidentMax = 1024;
  struct Resident {
    std::mutex mu;
    l7m::ResidentBox* box = nullptr;   // pinned host memory
    l7m::ResidentBox* dbox = nullptr;  // its device address
    hipStream_t stream = nullptr;
    uint32_t* qhdr = nullptr;          // device: the Kafka instantiations' queue counter
    hipEvent_t end = nullptr;          // recorded after the running instance
    bool running = false;
    uint64_t posted = 0;
    // programs the workgroup may still read, with the last sequence number
    // posted with each: released once done_seq has passed it (the workgroup
    // dereferences a slot's program only while it evaluates that slot)
    std::vector<std::pair<l7m_ruleset*, uint64_t>> held;
    l7m_ruleset* slot_rs[l7m::kResidentSlots] = {};  // rule set of each posted slot
    // per slot: the sequence number whose outcome its poster has read; a slot
    // is posted again only after that (result / stamps are not overwritten
    // under a poster that has not read them yet)
    std::atomic<uint64_t> consumed[l7m::kResidentSlots] = {};
    std::atomic<bool> ok{false};
  } res;
  // (res.mu held)
  void resident_hold_locked(l7m_ruleset* r, uint64_t seq) {
    for (auto& h : res.held)
      if (h.first == r) {
        h.second = std::max(h.second, seq);
        return;
      }
    l7m_retain(r);
    res.held.emplace_back(r, seq);
  }
  // (res.mu held) release programs no pending slot refers to
  void resident_trim_locked() {
    const uint64_t done = __atomic_load_n(&res.box->done_seq, __ATOMIC_ACQUIRE);
    size_t k = 0;
    for (auto& h : res.held) {
      if (h.second <= done) l7m_release(h.first);
      else res.held[k++] = h;
    }
    res.held.resize(k);
  }

  void resident_init() {
    (void)hipSetDevice(device);
    void* p = nullptr;
    if (hipHostMalloc(&p, sizeof(l7m::ResidentBox), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess || !p)
      return;
    std::memset(p, 0, sizeof(l7m::ResidentBox));
    res.box = static_cast<l7m::ResidentBox*>(p);
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d ||
        hipStreamCreateWithFlags(&res.stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&res.end, hipEventDisableTiming) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&res.qhdr), 16) != hipSuccess || hipMemset(res.qhdr, 0, 16) != hipSuccess)
      return;
    res.dbox = static_cast<l7m::ResidentBox*>(d);
    res.ok = !std::getenv("L7M_NO_RESIDENT");
  }
  void resident_fini() {
    if (res.box) {
      __atomic_store_n(&res.box->quit, 1ull, __ATOMIC_RELEASE);
      if (res.running && res.end) (void)hipEventSynchronize(res.end);
      if (res.running) l7m::resident_running(device, -1);
      res.running = false;
    }
    for (auto& h : res.held) l7m_release(h.first);
    res.held.clear();
    if (res.end) (void)hipEventDestroy(res.end);
    if (res.qhdr) (void)hipFree(res.qhdr);
    if (res.stream) (void)hipStreamDestroy(res.stream);
    if (res.box) (void)hipHostFree(res.box);
  }
  // (res.mu held) the running instance has ended: its cached programs may go
  void resident_reap_locked() {
    if (res.running && __atomic_load_n(&res.box->exited, __ATOMIC_ACQUIRE)) {  // it reads no program any more
      res.running = false;
      l7m::resident_running(device, -1);
      for (auto& h : res.held) l7m_release(h.first);
      res.held.clear();
    }
  }
  // (res.mu held) a workgroup for the oldest pending slot
  bool resident_launch_locked() {
    const uint64_t first = __atomic_load_n(&res.box->done_seq, __ATOMIC_ACQUIRE) + 1;
    if (first > res.posted) return true;
    const int kind = static_cast<int>(
        __atomic_load_n(&res.box->slots[first % l7m::kResidentSlots].kind, __ATOMIC_ACQUIRE));
    __atomic_store_n(&res.box->exited, 0ull, __ATOMIC_RELEASE);
    if (l7m::launch_resident(res.dbox, first, kind, res.qhdr, res.stream) != hipSuccess ||
        hipEventRecord(res.end, res.stream) != hipSuccess) {
      // no workgroup will take the posted slots: stop using the resident path
      // (their callers get L7M_EDEVICE; later batches are launched).  exited
      // goes back to 1 so flushers spinning on posted slots look again.
      res.ok = false;
      __atomic_store_n(&res.box->exited, 1ull, __ATOMIC_RELEASE);
      return false;
    }
    res.running = true;
    l7m::resident_running(device, 1);
    for (uint64_t q = first; q <= res.posted; ++q) resident_hold_locked(res.slot_rs[q % l7m::kResidentSlots], q);
    return true;
  }
  // Evaluate batch b (cnt records, bytes) on the resident workgroup.
  int resident_eval(l7m_ruleset* r, const uint32_t* dprog, int kind, uint32_t stage, uint64_t serial, Batch* b,
                    uint32_t cnt, uint64_t bytes) {
    uint64_t seq;
    {
      std::unique_lock<std::mutex> lk(res.mu);
      // ring full (more flushers than slots), or the slot's previous poster
      // has not read its outcome yet: let them catch up
      while (res.posted - __atomic_load_n(&res.box->done_seq, __ATOMIC_ACQUIRE) >= l7m::kResidentSlots ||
             (res.posted + 1 > l7m::kResidentSlots &&
              res.consumed[(res.posted + 1) % l7m::kResidentSlots].load(std::memory_order_acquire) <
                  res.posted + 1 - l7m::kResidentSlots)) {
        if (!res.ok) return 1;  // the resident path was turned off meanwhile: normal launches
        lk.unlock();
        cpu_relax();
        lk.lock();
      }
      if (!res.ok) return 1;
      seq = ++res.posted;
      l7m::ResidentSlot& sl = res.box->slots[seq % l7m::kResidentSlots];
      auto put = [](uint64_t* f, uint64_t v) { __atomic_store_n(f, v, __ATOMIC_RELAXED); };
      put(&sl.kind, static_cast<uint64_t>(kind));
      put(&sl.gen, serial);
      put(&sl.prog, reinterpret_cast<uint64_t>(dprog));
      put(&sl.arena, reinterpret_cast<uint64_t>(b->d_arena));
      put(&sl.arena_bytes, bytes);
      put(&sl.offs, reinterpret_cast<uint64_t>(b->d_offs));
      put(&sl.n, cnt);
      put(&sl.verdicts, reinterpret_cast<uint64_t>(b->d_verd));
      put(&sl.stage, stage);
      put(&sl.ids, reinterpret_cast<uint64_t>(b->d_ids));
      put(&sl.result, 0);
      for (uint64_t& x : sl.stamp) put(&x, 0);
      res.slot_rs[seq % l7m::kResidentSlots] = r;
      resident_trim_locked();
      resident_hold_locked(r, seq);
      __atomic_store_n(&res.box->post_seq, seq, __ATOMIC_RELEASE);
      resident_reap_locked();
      if (!res.running && !resident_launch_locked()) return L7M_EDEVICE;
    }
    // L7M_OK, or 1: the workgroup asks for the normal launches (Kafka
    // batches with compressed message sets need the codec pass)
    auto outcome = [&]() -> int {
      const l7m::ResidentSlot& sl = res.box->slots[seq % l7m::kResidentSlots];
      uint64_t st[4];
      for (int k = 0; k < 4; ++k) st[k] = __atomic_load_n(&sl.stamp[k], __ATOMIC_ACQUIRE);
      if (st[0] && st[3] >= st[2] && st[2] >= st[1] && st[1] >= st[0]) {
        res_batches.fetch_add(1);
        res_read.fetch_add(st[1] - st[0]);
        res_eval.fetch_add(st[2] - st[1]);
        res_sync.fetch_add(st[3] - st[2]);
      }
      const int out = __atomic_load_n(&sl.result, __ATOMIC_ACQUIRE) ? 1 : L7M_OK;
      res.consumed[seq % l7m::kResidentSlots].store(seq, std::memory_order_release);  // the slot may be posted again
      return out;
    };
    for (uint32_t spin = 0;; ++spin) {
      if (__atomic_load_n(&res.box->done_seq, __ATOMIC_ACQUIRE) >= seq) return outcome();
      if ((spin & 63) == 63 && (__atomic_load_n(&res.box->exited, __ATOMIC_ACQUIRE) || !res.ok)) {
        // idle exit / other kind / a failed launch
        std::lock_guard<std::mutex> g(res.mu);
        if (__atomic_load_n(&res.box->done_seq, __ATOMIC_ACQUIRE) >= seq) return outcome();
        if (!res.ok) return L7M_EDEVICE;  // no workgroup will take this slot
        resident_reap_locked();
        if (!res.running && !resident_launch_locked()) return L7M_EDEVICE;
      }
      cpu_relax();
    }
  }

  Batch* fresh() {
    {
      std::lock_guard<std::mutex> g(pool_mu);
      if (!pool.empty()) {
        Batch* b = pool.back();
        pool.pop_back();
        b->reset();
        return b;
      }
    }
    auto* b = new (std::nothrow) Batch();
    if (!b) return nullptr;
    (void)hipSetDevice(device);
    if (!b->alloc(arena_cap, max_batch)) {
      delete b;
      return nullptr;
    }
    std::lock_guard<std::mutex> g(pool_mu);
    all.push_back(b);
    return b;
  }
  void recycle(Batch* b) {
    std::lock_guard<std::mutex> g(pool_mu);
    pool.push_back(b);
  }
  void wake_flusher() {
    if (idle.load() == 0) return;
    std::lock_guard<std::mutex> g(idle_mu);
    idle_cv.notify_one();
  }

  // Per-batch bookkeeping once its verdicts are in (or its launch failed).
  void finish(Batch* b, l7m_ruleset* r, uint32_t cnt, int rc, int64_t t_close, int64_t t_launch) {
    const int64_t t_done = now_ns();
    l7m_release(r);
    batches.fetch_add(1);
    requests.fetch_add(cnt);
    const int64_t t_first = b->first_ns.load();
    if (t_first > 0 && t_close > t_first) {  // a batch without its stamp is left out of the fill phase
      fill_ns.fetch_add(static_cast<uint64_t>(t_close - t_first));
      fill_batches.fetch_add(1);
    }
    launch_ns.fetch_add(static_cast<uint64_t>(t_launch - t_close));
    gpu_ns.fetch_add(static_cast<uint64_t>(t_done - t_launch));
    b->rc = rc;
    b->done_ns = t_done;
    b->readers.store(cnt);
    b->done.store(1);  // seq_cst with the callers' sleepers increment (no lost wake-up)
    if (b->sleepers.load()) {
      std::lock_guard<std::mutex> g(b->m);
      b->cv.notify_all();
    }
  }

  // A flusher keeps up to `pipe` kernel-signalled HTTP launches in flight,
  // one per slot (own stream, own completion word), and goes back to the
  // fill while they run; pipe 1 waits for each launch before the next batch.
  struct Slot {
    hipStream_t stream = nullptr;
    uint32_t* ctr = nullptr;   // device: the kernel's wave counter
    uint32_t* host = nullptr;  // pinned: the completion word
    void* dev = nullptr;       // its device address
    uint32_t seq = 0;
    bool busy = false;
    Batch* b = nullptr;
    l7m_ruleset* r = nullptr;
    uint32_t cnt = 0, spins = 0;
    int64_t t_close = 0, t_launch = 0;
  };
  uint32_t pipe = 1;

  void run() {
    (void)hipSetDevice(device);
    hipEvent_t ev = nullptr;
    std::vector<Slot> slots(pipe);
    bool dev_ok = hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess;
    // HTTP launches signal their completion by a pinned host word the kernel
    // stores last (l7m_device.h DoneSignal): polled in place of an event,
    // whose completion the host sees only after the command processor's
    // end-of-kernel signal
    bool sig_ok = dev_ok;
    for (Slot& q : slots) {
      dev_ok = dev_ok && hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking) == hipSuccess;
      sig_ok = sig_ok && dev_ok && hipMalloc(reinterpret_cast<void**>(&q.ctr), 64) == hipSuccess &&
               hipMemset(q.ctr, 0, 64) == hipSuccess &&
               hipHostMalloc(reinterpret_cast<void**>(&q.host), 64, hipHostMallocMapped | hipHostMallocCoherent) ==
                   hipSuccess &&
               hipHostGetDevicePointer(&q.dev, q.host, 0) == hipSuccess && q.dev;
      if (q.host) std::memset(q.host, 0, 64);
    }
    sig_ok = sig_ok && dev_ok;
    if (std::getenv("L7M_NO_SIGNAL")) sig_ok = false;
    hipStream_t stream = slots[0].stream;  // unsignalled launches (after the slots have drained)
    uint32_t npending = 0;
    // Completes the in-flight launches whose word has arrived (all of them
    // when `all`); the stream is checked now and then so that a failed launch
    // cannot leave a slot pending.
    auto poll = [&](bool all) {
      for (;;) {
        for (Slot& q : slots) {
          if (!q.busy) continue;
          int rc = L7M_OK;
          bool done = __atomic_load_n(q.host, __ATOMIC_ACQUIRE) == q.seq;
          if (!done && (++q.spins & 1023) == 0) {
            const hipError_t e = hipStreamQuery(q.stream);
            if (e != hipErrorNotReady) {
              done = true;
              if (e != hipSuccess || __atomic_load_n(q.host, __ATOMIC_ACQUIRE) != q.seq) rc = L7M_EDEVICE;
            }
          }
          if (!done) continue;
          q.busy = false;
          --npending;
          finish(q.b, q.r, q.cnt, rc, q.t_close, q.t_launch);
        }
        if (!all || npending == 0) return;
        cpu_relax();
      }
    };
    for (;;) {
      if (npending) poll(false);
      Batch* b = cur.load(std::memory_order_acquire);
      const uint64_t s0 = b->resv.load(std::memory_order_acquire);
      const uint32_t cnt0 = count_of(s0);
      if (cnt0 == 0) {
        if (npending) {  // launches in flight: keep polling them
          cpu_relax();
          continue;
        }
        if (stop.load()) break;
        // idle: poll a little, then sleep until a caller's first append
        const int64_t t0 = now_ns();
        bool work = false;
        while (now_ns() - t0 < 100000) {  // 100 us: a busy proxy's next request usually comes sooner
          if (count_of(cur.load(std::memory_order_acquire)->resv.load(std::memory_order_acquire)) || stop.load()) {
            work = true;
            break;
          }
          cpu_relax();
        }
        if (!work) {
          std::unique_lock<std::mutex> lk(idle_mu);
          idle.fetch_add(1);
          if (!count_of(cur.load()->resv.load()) && !stop.load())
            idle_cv.wait_for(lk, std::chrono::milliseconds(2));
          idle.fetch_sub(1);
        }
        continue;
      }
      const int64_t first = b->first_ns.load();  // 0 until the first caller has stamped it
      // Deadline mode flushes at max_batch, a full arena, max_delay_us after the
      // first request -- or as soon as every caller inside l7m_batcher_eval that
      // is not already waiting on an evaluated batch is in this one: nobody is
      // left to join it, so waiting out the deadline would only add latency.
      // A hint, not a snapshot: in_closed is read before callers, so a batch
      // closed or a caller arriving between the two loads makes the estimate
      // larger, i.e. errs toward waiting.
      const int64_t closed_now = in_closed.load();
      const int64_t free_callers = static_cast<int64_t>(callers.load()) - closed_now;
      if (!eager && !stop.load() && cnt0 < max_batch && !b->want_close.load() && static_cast<int64_t>(cnt0) < free_callers &&
          (first == 0 || now_ns() - first < static_cast<int64_t>(max_delay_us) * 1000)) {
        cpu_relax();
        continue;
      }
      if (npending == pipe) {  // every slot in flight: this batch waits for one
        cpu_relax();
        continue;
      }
      uint64_t s;
      {
        std::lock_guard<std::mutex> g(close_mu);
        // another flusher took it; or b was taken, recycled and is current again
        // but still empty (s0 came from its previous use): closing it would
        // evaluate nothing and strand the batch outside the pool
        if (cur.load() != b || count_of(b->resv.load()) == 0) continue;
        Batch* nb = fresh();
        if (!nb) {  // out of pinned memory: evaluate what is there, keep filling b's successor later
          std::this_thread::sleep_for(std::chrono::microseconds(100));
          continue;
        }
        s = b->resv.fetch_or(kClosed);
        cur.store(nb, std::memory_order_release);
        in_closed.fetch_add(count_of(s));
      }
      const uint32_t cnt = count_of(s);
      const uint64_t bytes = bytes_of(s);
      const int64_t t_close = now_ns();
      while (b->written.load(std::memory_order_acquire) < cnt) cpu_relax();
      l7m_ruleset* r;
      {
        std::lock_guard<std::mutex> g(rs_mu);
        r = rs;
        l7m_retain(r);
      }
      l7m_ruleset_info info;
      l7m_ruleset_get_info(r, &info);
      int rc = dev_ok ? L7M_OK : L7M_EDEVICE;
      const uint32_t* dprog = nullptr;
      int kind = 0;
      uint32_t stage = 0;
      uint64_t serial = 0;
      int64_t t_launch = t_close;
      bool normal = true;
      if (rc == L7M_OK && res.ok && cnt <= kResidentMax &&
          l7m::resident_program(r, &dprog, &kind, &stage, &serial)) {
        t_launch = now_ns();
        rc = resident_eval(r, dprog, kind, stage, serial, b, cnt, bytes);
        normal = rc == 1;
        if (normal) rc = L7M_OK;
      }
      if (normal) {
        bool signalled = false;
        if (rc == L7M_OK && info.proto == L7M_PROTO_HTTP && sig_ok) {
          Slot* q = nullptr;
          for (Slot& x : slots)
            if (!x.busy) {
              q = &x;
              break;
            }
          // (npending < pipe above: a slot is free)
          if (!++q->seq) ++q->seq;
          const l7m::DoneSignal sg{q->ctr, static_cast<uint32_t*>(q->dev), q->seq};
          rc = l7m::eval_device_signal(r, b->d_arena, bytes, b->d_offs, cnt, b->d_verd, q->stream, sg, &signalled);
          t_launch = now_ns();
          if (rc == L7M_OK && signalled) {
            // the kernel's deciding wave stores q->seq after every verdict is
            // visible (l7m_device.h DoneSignal); poll() completes the batch
            q->busy = true;
            q->b = b;
            q->r = r;
            q->cnt = cnt;
            q->spins = 0;
            q->t_close = t_close;
            q->t_launch = t_launch;
            ++npending;
            if (npending == pipe) poll(false);
            continue;
          }
          stream = q->stream;
        } else if (rc == L7M_OK) {
          poll(true);  // unsignalled launches wait for an event: no slot in flight meanwhile
          stream = slots[0].stream;
          rc = info.proto == L7M_PROTO_KAFKA
                   ? l7m_eval_device_ids(r, b->d_arena, bytes, b->d_offs, cnt, b->d_ids, b->d_verd, nullptr, stream, 0)
                   : l7m_eval_device(r, b->d_arena, bytes, b->d_offs, cnt, b->d_verd, nullptr, stream, 0);
          t_launch = now_ns();
        }
        if (rc == L7M_OK && hipEventRecord(ev, stream) != hipSuccess) rc = L7M_EDEVICE;
        if (rc == L7M_OK) {
          hipError_t e;
          while ((e = hipEventQuery(ev)) == hipErrorNotReady) cpu_relax();
          if (e != hipSuccess) rc = L7M_EDEVICE;
        }
      }
      finish(b, r, cnt, rc, t_close, t_launch);
    }
    poll(true);
    for (Slot& q : slots) {
      if (q.stream) (void)hipStreamSynchronize(q.stream);
      if (q.ctr) (void)hipFree(q.ctr);
      if (q.host) (void)hipHostFree(q.host);
      if (q.stream) (void)hipStreamDestroy(q.stream);
    }
    if (ev) (void)hipEventDestroy(ev);
  }

  // A record that can never fit a batch: evaluated alone (copying path).
  int eval_alone(const uint8_t* rec, size_t len, uint32_t src_identity, int32_t* verdict) {
    l7m_ruleset* r;
    {
      std::lock_guard<std::mutex> g(rs_mu);
      r = rs;
      l7m_retain(r);
    }
    std::vector<uint8_t> a((len + 3 + 64) & ~size_t(3), 0);
    if (len) std::memcpy(a.data(), rec, len);
    const uint64_t off = 0;
    (void)hipSetDevice(device);
    l7m_ruleset_info info;
    l7m_ruleset_get_info(r, &info);
    const int rc = l7m_eval_ids(r, a.data(), (len + 3) & ~size_t(3), &off, 1,
                                info.proto == L7M_PROTO_KAFKA ? &src_identity : nullptr, verdict, nullptr, 0);
    l7m_release(r);
    return rc;
  }

  int eval(const uint8_t* rec, size_t len, uint32_t src_identity, int32_t* verdict) {
    if (stop.load()) return L7M_EINVAL;
    callers.fetch_add(1);
    if (stop.load()) {
      callers.fetch_sub(1);
      return L7M_EINVAL;
    }
    const size_t padded = (len + 3) & ~size_t(3);
    if (padded > arena_cap) {
      const int rc = eval_alone(rec, len, src_identity, verdict);
      callers.fetch_sub(1);
      return rc;
    }
    // reserve a slot and its bytes in the batch being filled
    Batch* b;
    uint32_t idx;
    uint64_t off;
    const int64_t t_arrive = now_ns();  // stamped before the reservation, so never after the close
    for (;;) {
      b = cur.load(std::memory_order_acquire);
      uint64_t s = b->resv.load(std::memory_order_acquire);
      if (s & kClosed) {
        cpu_relax();
        continue;
      }
      const uint32_t cnt = count_of(s);
      if (cnt >= b->cap || bytes_of(s) + padded > b->arena_cap) {  // full: the flusher takes it
        b->want_close.store(1);
        wake_flusher();
        cpu_relax();
        continue;
      }
      if (b->resv.compare_exchange_weak(s, s + (1ull << kCountShift) + padded, std::memory_order_acq_rel)) {
        idx = cnt;
        off = bytes_of(s);
        break;
      }
    }
    if (idx == 0) b->first_ns.store(t_arrive);
    if (len) std::memcpy(b->arena + off, rec, len);
    if (padded != len) std::memset(b->arena + off + len, 0, padded - len);
    b->offs[idx] = off;
    b->ids[idx] = src_identity;
    b->written.fetch_add(1, std::memory_order_release);
    if (idx == 0 || idx + 1 >= max_batch) wake_flusher();
    // wait for the verdict: spin, then sleep
    const int64_t t0 = now_ns();
    uint32_t spins = 0;
    while (!b->done.load(std::memory_order_acquire)) {
      if ((++spins & 63) == 0 && now_ns() - t0 > kSpinNs) {
        b->sleepers.fetch_add(1);
        std::unique_lock<std::mutex> lk(b->m);
        b->cv.wait(lk, [&] { return b->done.load() != 0; });
        b->sleepers.fetch_sub(1);
        break;
      }
      cpu_relax();
    }
    const int rc = b->rc;
    if (rc == L7M_OK) *verdict = b->verd[idx];
    in_closed.fetch_sub(1);
    wake_ns.fetch_add(static_cast<uint64_t>(now_ns() - b->done_ns));
    if (b->readers.fetch_sub(1) == 1) recycle(b);  // the last reader recycles the batch
    callers.fetch_sub(1);
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
  // arena of a batch: about 256 bytes per request, 1-16 MiB
  const size_t want = static_cast<size_t>(b->max_batch) * 256u;
  b->arena_cap = want < (1u << 20) ? (1u << 20) : want > (16u << 20) ? (16u << 20) : want;
  Batch* first = b->fresh();
  if (!first) {
    delete b;
    return L7M_ENOMEM;
  }
  b->cur.store(first);
  l7m_retain(rs);
  b->rs = rs;
  b->resident_init();
  if (const char* e = std::getenv("L7M_PIPE")) {  // (experiment) launches in flight per flusher
    const int v = std::atoi(e);
    b->pipe = v < 1 ? 1u : v > 4 ? 4u : static_cast<uint32_t>(v);
  }
  for (uint32_t i = 0; i < b->in_flight; ++i) b->flushers.emplace_back([b] { b->run(); });
  *out = b;
  return L7M_OK;
}

int l7m_batcher_set_ruleset(l7m_batcher* b, l7m_ruleset* rs) {
  if (!b || !rs) return L7M_EINVAL;
  l7m_retain(rs);
  l7m_ruleset* old;
  {
    std::lock_guard<std::mutex> lk(b->rs_mu);
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
  if (batches) *batches = b->batches.load();
  if (requests) *requests = b->requests.load();
  return L7M_OK;
}

int l7m_batcher_get_profile(l7m_batcher* b, l7m_batcher_profile* out) {
  if (!b || !out) return L7M_EINVAL;
  const uint64_t nb = b->batches.load(), nr = b->requests.load();
  out->batches = nb;
  out->requests = nr;
  const uint64_t nf = b->fill_batches.load();
  out->fill_us = nf ? b->fill_ns.load() / 1e3 / nf : 0.0;
  out->launch_us = nb ? b->launch_ns.load() / 1e3 / nb : 0.0;
  out->gpu_us = nb ? b->gpu_ns.load() / 1e3 / nb : 0.0;
  const uint64_t rb = b->res_batches.load();
  out->resident_batches = rb;
  out->resident_rounds = b->res.box ? __atomic_load_n(&b->res.box->rounds, __ATOMIC_ACQUIRE) : 0;
  out->resident_read_us = rb ? b->res_read.load() / 100.0 / rb : 0.0;  // 100 ticks per us
  out->resident_eval_us = rb ? b->res_eval.load() / 100.0 / rb : 0.0;
  out->resident_sync_us = rb ? b->res_sync.load() / 100.0 / rb : 0.0;
  out->wake_us = nr ? b->wake_ns.load() / 1e3 / nr : 0.0;
  return L7M_OK;
}

// Safe with calls in flight: pending batches are still evaluated, new calls
// get L7M_EINVAL, and the batcher is freed only after every caller inside
// l7m_batcher_eval* has read its verdict and left.
void l7m_batcher_destroy(l7m_batcher* b) {
  if (!b) return;
  b->stop.store(true);
  {
    std::lock_guard<std::mutex> g(b->idle_mu);
    b->idle_cv.notify_all();
  }
  // callers already inside finish their reservation; flushers drain the
  // pending batches and exit once the current batch stays empty
  while (b->callers.load() != 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
  for (auto& t : b->flushers)
    if (t.joinable()) t.join();
  b->resident_fini();
  l7m_release(b->rs);
  for (Batch* x : b->all) delete x;
  delete b;
}

}  // extern "C"
