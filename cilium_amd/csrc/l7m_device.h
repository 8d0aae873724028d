// l7m_device.h — launch entry points of the HIP kernels (l7m_kernels.hip,
// l7m_kafka.hip) used by the C ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

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
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  std::lock_guard<std::mutex> g(mu);
  if (done.count({fn, dev})) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
  if (e == hipSuccess) done.insert({fn, dev});
  return e;
}

// LDS bytes of one HTTP workgroup with `stage` bytes of records per wave, and
// the stage the LDS leaves after the rule tables (0: the tables do not fit).
size_t http_lds_bytes(const HttpHeader& h, uint32_t stage);
uint32_t http_stage_bytes(const HttpHeader& h);
// Internal launch flag (beside the public L7M_FLAG_* bits): the program has
// literal tables (DfaDesc::lit_tab), so the kernel instantiation that uses
// them is launched.
constexpr uint32_t kLaunchLiterals = 1u << 29;  // L7M_FLAG_DIAG_* use bits 30, 31
hipError_t launch_http(const uint32_t* dprog, const HttpHeader& h, const uint8_t* arena,
                       uint64_t arena_bytes, const uint64_t* offs, uint64_t n, int32_t* verdicts,
                       unsigned long long* hits, hipStream_t stream, int num_cus, uint32_t flags);

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
