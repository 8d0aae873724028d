// l7m_device.h — launch entry points of the HIP kernels (l7m_kernels.hip,
// l7m_kafka.hip) used by the C ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <utility>

#include "program.h"

namespace l7m {

// Raise a kernel's dynamic-LDS limit (gfx950: up to 160 KiB per workgroup)
// once per (kernel, device), thread-safely: l7m_eval is reentrant and a rule
// set may be evaluated on several devices.  Returns the HIP status.
inline hipError_t set_lds_attr_once(const void* fn, uint32_t bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  // per-thread cache of the (kernel, device) pairs already done: the
  // batcher's flushers launch per batch and would contend on the mutex
  static thread_local const void* last_fn = nullptr;
  static thread_local int last_dev = -1;
  if (fn == last_fn && dev == last_dev) return hipSuccess;
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  std::lock_guard<std::mutex> g(mu);
  if (!done.count({fn, dev})) {
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
    if (e != hipSuccess) return e;
    done.insert({fn, dev});
  }
  last_fn = fn;
  last_dev = dev;
  return hipSuccess;
}

// Stream-ordered scratch (the slow pass's executor stacks, the search
// programs' code columns) comes from a PRIVATE memory pool per device, so
// the embedding process's default pool (its own hipMallocAsync behaviour) is
// left alone.  The private pool keeps up to 2 GiB mapped between
// launches instead of returning it at every synchronisation.  Falls back to
// the default pool (hipMallocAsync) if the runtime refuses to create one.
// Free with hipFreeAsync on the base pointer.
inline hipError_t scratch_alloc_async(void** p, size_t bytes, hipStream_t stream) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  static std::mutex mu;
  static std::map<int, hipMemPool_t> pools;
  hipMemPool_t pool = nullptr;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = pools.find(dev);
    if (it == pools.end()) {
      hipMemPoolProps props;
      std::memset(&props, 0, sizeof props);
      props.allocType = hipMemAllocationTypePinned;
      props.handleTypes = hipMemHandleTypeNone;
      props.location.type = hipMemLocationTypeDevice;
      props.location.id = dev;
      if (hipMemPoolCreate(&pool, &props) == hipSuccess && pool) {
        uint64_t keep = 2ull << 30;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
      } else {
        pool = nullptr;
        (void)hipGetLastError();
      }
      pools[dev] = pool;  // nullptr: use the default pool
    } else {
      pool = it->second;
    }
  }
  return pool ? hipMallocFromPoolAsync(p, bytes, pool, stream) : hipMallocAsync(p, bytes, stream);
}

// LDS bytes of one HTTP workgroup with `stage` bytes of records per wave, and
// the stage the LDS leaves after the rule tables (0: the tables do not fit).
size_t http_lds_bytes(const HttpHeader& h, uint32_t stage);
uint32_t http_stage_bytes(const HttpHeader& h);
// Internal launch flag (beside the public L7M_FLAG_* bits): the program has
// literal tables (DfaDesc::lit_tab), so the kernel instantiation that uses
// them is launched.
constexpr uint32_t kLaunchLiterals = 1u << 29;  // L7M_FLAG_DIAG_* use bits 30, 31
// Completion signal of a first-pass launch (the batcher's latency path):
// every wave, once its verdicts are visible system-wide, adds one to *ctr
// (device memory, zero between launches); the last one resets it and stores
// seq to *flag (pinned host memory, system scope), which the host polls
// instead of a HIP event.  Only for programs decided in one launch (no slow
// pass).
struct DoneSignal {
  uint32_t* ctr;
  uint32_t* flag;
  uint32_t seq;
};
hipError_t launch_http(const uint32_t* dprog, const HttpHeader& h, const uint8_t* arena,
                       uint64_t arena_bytes, const uint64_t* offs, uint64_t n, int32_t* verdicts,
                       unsigned long long* hits, hipStream_t stream, int num_cus, uint32_t flags,
                       const DoneSignal* done = nullptr);

// Mailbox of a resident evaluator (l7m_kafka.hip kafka_resident_kernel),
// in pinned, device-mapped host memory.  The host fills slot seq %
// kResidentSlots, then raises post_seq to seq (release); the workgroup
// evaluates the slot and raises done_seq to seq.  Every field is read and
// written with system-scope atomics.
constexpr uint32_t kResidentSlots = 16;
constexpr uint32_t kResidentRound = 16;      // slots one resident round evaluates together (one per wave at most)
constexpr uint32_t kResidentLdsWords = 2 * (4 + 16 * kResidentRound);  // broadcast words at the end of its LDS
constexpr uint64_t kResidentIdleTicks = 2000000;  // 20 ms of s_memrealtime (100 MHz) without work: exit
constexpr uint64_t kResidentKafka = 16;          // kind of a Kafka slot: kResidentKafka | cli_lds | groups << 1
struct ResidentSlot {
  uint64_t kind;  // the instantiation: kResidentKafka | cli_lds | groups << 1
  uint64_t gen;   // program generation (a new program at a reused address reloads the image)
  uint64_t prog, arena, arena_bytes, offs, n, verdicts, stage, ids;
  uint64_t result;  // written by the workgroup: 1 = evaluate this batch again with the normal launches
  // written by the workgroup (s_memrealtime, 100 MHz): batch seen, slot read
  // and caches invalidated, batch evaluated, verdicts written back
  uint64_t stamp[4];
  uint64_t pad;
};
static_assert(sizeof(ResidentSlot) == 128, "the resident workgroup reads a slot as 16 words");
struct ResidentBox {
  alignas(64) uint64_t post_seq;
  alignas(64) uint64_t done_seq;
  alignas(64) uint64_t quit;
  alignas(64) uint64_t exited;  // set by the workgroup as it returns (cleared by the host before a launch)
  alignas(64) uint64_t rounds;  // rounds evaluated (statistics)
  alignas(64) ResidentSlot slots[kResidentSlots];
};
// Whether a Kafka program can be served by the resident evaluator, with
// which instantiation and record stage.
bool kafka_resident_ok(const KafkaHeader& h, int* kind, uint32_t* stage);
// Launch the resident workgroup of `kind` for slots first_seq, ...; qhdr: 16
// bytes of zeroed device memory (the Kafka instantiations' queue counter).
hipError_t launch_resident(ResidentBox* dbox, uint64_t first_seq, int kind, uint32_t* qhdr, hipStream_t stream);
hipError_t launch_kafka_resident(ResidentBox* dbox, uint64_t first_seq, int kind, uint32_t* qhdr,
                                 hipStream_t stream);

// Device scratch of the Kafka path's compressed-message second pass: the
// queue of request indices the first pass fills (header [0] pushed, [1] work
// counter, zeroed before each launch) and `workers` slabs of slab_bytes for
// decoded sets.
struct KafkaCodecQueue {
  uint32_t* recs = nullptr;
  uint32_t* qhdr = nullptr;
  uint32_t cap = 0;      // 0: every request with a compressed message reports -3
  uint32_t workers = 0;
  uint8_t* slabs = nullptr;
  uint64_t slab_bytes = 0;
};

hipError_t launch_kafka(const uint32_t* dprog, const KafkaHeader& h, const uint8_t* arena,
                        uint64_t arena_bytes, const uint64_t* offs, uint64_t n, int32_t* verdicts,
                        unsigned long long* hits, hipStream_t stream, int num_cus, uint32_t flags,
                        const KafkaCodecQueue& cq, const uint32_t* ids);
hipError_t launch_kafka_codec(const uint32_t* dprog, const uint8_t* arena, uint64_t arena_bytes, const uint64_t* offs,
                              uint64_t n, int32_t* verdicts, unsigned long long* hits, hipStream_t stream,
                              const KafkaCodecQueue& cq);

}  // namespace l7m
