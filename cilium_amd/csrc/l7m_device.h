// l7m_device.h — launch entry points of the HIP kernels (l7m_kernels.hip,
// l7m_kafka.hip) used by the C ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "program.h"

namespace l7m {

// LDS bytes of one HTTP workgroup with `stage` bytes of records per wave, and
// the stage the LDS leaves after the rule tables (0: the tables do not fit).
size_t http_lds_bytes(const HttpHeader& h, uint32_t stage);
uint32_t http_stage_bytes(const HttpHeader& h);
hipError_t launch_http(const uint32_t* dprog, const HttpHeader& h, const uint8_t* arena,
                       uint64_t arena_bytes, const uint64_t* offs, uint64_t n, int32_t* verdicts,
                       unsigned long long* hits, hipStream_t stream, int num_cus, uint32_t flags);

hipError_t launch_kafka(const uint32_t* dprog, const KafkaHeader& h, const uint8_t* arena,
                        uint64_t arena_bytes, const uint64_t* offs, uint64_t n, int32_t* verdicts,
                        unsigned long long* hits, hipStream_t stream, int num_cus, uint32_t flags);

}  // namespace l7m
