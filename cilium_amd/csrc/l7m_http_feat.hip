// l7m_http_feat.hip -- the ECMAScript first-pass (http_eval_kernel) and
// slow-pass (http_slow_kernel) instantiations of ONE feature set, kFeat =
// L7M_FEAT (l7m_http_impl.h kFeatLit / kFeatDcap).  Compiled once per feature
// set (Makefile: build/l7m_http_f<F>.o), so the instantiations build in
// parallel; l7m_kernels.hip launch_http picks the set a program needs.
#include "l7m_http_impl.h"

#ifndef L7M_FEAT
#error "L7M_FEAT (0..3) selects the feature set"
#endif
#define L7M_CAT2(a, b) a##b
#define L7M_CAT(a, b) L7M_CAT2(a, b)

namespace l7m {

hipError_t L7M_CAT(launch_http_main_f, L7M_FEAT)(int mode, int R, dim3 grid, size_t lds, hipStream_t stream,
                                                 const uint32_t* dprog, const uint8_t* arena, uint64_t arena_bytes,
                                                 const uint64_t* offs, uint64_t n, int32_t* verdicts,
                                                 unsigned long long* hits, uint32_t stage, uint32_t* slowq,
                                                 DoneSignal done, uint32_t* hslice) {
#define L7M_ONE(M, RR)                                                                                       \
  return launch_one<M, RR, 0, L7M_FEAT>(grid, lds, stream, dprog, arena, arena_bytes, offs, n, verdicts, hits, \
                                        stage, nullptr, slowq, done, hslice)
#define L7M_MODES(RR)                             \
  {                                               \
    if (mode == kNoHits) L7M_ONE(kNoHits, RR);    \
    if (mode == kLdsHits) L7M_ONE(kLdsHits, RR);  \
    L7M_ONE(kGlobalHits, RR);                     \
  }
  if (R == 4) L7M_MODES(4)
  if (R == 8) L7M_MODES(8)
  L7M_MODES(0)
#undef L7M_MODES
#undef L7M_ONE
}

hipError_t L7M_CAT(launch_http_slow_f, L7M_FEAT)(int R, int tier, const HttpHeader& h, uint32_t blocks,
                                                 hipStream_t stream, const uint32_t* dprog, const uint8_t* arena,
                                                 uint64_t arena_bytes, const uint64_t* offs, uint64_t n,
                                                 int32_t* verdicts, unsigned long long* hits, const uint32_t* slowq,
                                                 uint32_t* slowq2, uint32_t* vmscratch, uint32_t* work) {
#define L7M_SLOW(RR, T)                                                                                          \
  return launch_slow<RR, L7M_FEAT, T>(h, blocks, stream, dprog, arena, arena_bytes, offs, n, verdicts, hits, slowq, \
                                      slowq2, vmscratch, work)
  if (tier == 1) {
    if (R == 4) L7M_SLOW(4, 1);
    if (R == 8) L7M_SLOW(8, 1);
    L7M_SLOW(0, 1);
  }
  if (R == 4) L7M_SLOW(4, 2);
  if (R == 8) L7M_SLOW(8, 2);
  L7M_SLOW(0, 2);
#undef L7M_SLOW
}

}  // namespace l7m
