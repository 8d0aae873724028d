// l7m_kernels.hip — CDNA4 (gfx950) kernel of the batched HTTP verdict path.
//
// Persistent layout: one 1024-thread workgroup (16 waves) per CU.  Each wave
// owns a contiguous range of the batch and consumes it in tiles of up to 64
// consecutive records (one lane per record):
//   1. the tile's byte window [off_first, end_last) is copied HBM -> the
//      wave's LDS stage with coalesced 16-byte non-temporal loads (the arena is
//      streamed exactly once; the tile is cut short so the window fits);
//   2. walk phase: every referenced field (method / path / authority / values
//      of headers whose lower-cased name a rule references) is walked through
//      its packed DFA groups (dfa_pack.h) in one loop of walk jobs: one
//      dependent 4-byte LDS read per input byte, tables copied to LDS once per
//      workgroup;
//   3. the next tile's bytes are requested;
//   4. verification phase: the end codes select precomputed candidate rule
//      lists (L2-resident); the first rule (input order) whose other
//      matchers hold is the verdict.
// A record that is not inside its tile window (non-contiguous offsets, a
// record larger than the stage, malformed lengths) is evaluated by the same
// code reading HBM directly.
// Reference semantics: NetworkPolicyMap::Allowed -> PortNetworkPolicyRule::
// Matches -> HttpNetworkPolicyRule::Matches -> ConfigUtility::matchHeaders
// (envoy/cilium_network_policy.h:68-237).
#include "l7m_http_impl.h"

namespace l7m {

// First-pass / slow-pass launches of the ECMAScript instantiations of one
// feature set (l7m_http_feat.hip, compiled once per kFeat)
#define L7M_FEAT_DECL(F)                                                                                            \
  hipError_t launch_http_main_f##F(int mode, int R, dim3 grid, size_t lds, hipStream_t stream, const uint32_t* dprog,  \
                                   const uint8_t* arena, uint64_t arena_bytes, const uint64_t* offs, uint64_t n,        \
                                   int32_t* verdicts, unsigned long long* hits, uint32_t stage, uint32_t* slowq,       \
                                   DoneSignal done, uint32_t* hslice);                                                 \
  hipError_t launch_http_slow_f##F(int R, int tier, const HttpHeader& h, uint32_t blocks, hipStream_t stream,         \
                                   const uint32_t* dprog, const uint8_t* arena, uint64_t arena_bytes,                  \
                                   const uint64_t* offs, uint64_t n, int32_t* verdicts, unsigned long long* hits,      \
                                   const uint32_t* slowq, uint32_t* slowq2, uint32_t* vmscratch, uint32_t* work);
L7M_FEAT_DECL(0)
L7M_FEAT_DECL(1)
L7M_FEAT_DECL(2)
L7M_FEAT_DECL(3)
#undef L7M_FEAT_DECL

size_t http_lds_bytes(const HttpHeader& h, uint32_t stage) {
  const bool reg = h.n_dfas <= kRegDfas || h.search;  // search programs: codes in global scratch
  const size_t ctr = !kSliceHits && h.n_rules + 2 <= kMaxLdsCounters ? ((h.n_rules + 2 + 3) & ~size_t(3)) : 0;
  return 4u * (static_cast<size_t>(h.lds_image_words) + ctr + (reg ? 0u : static_cast<size_t>(h.n_dfas) * kBlock)) +
         static_cast<size_t>(kWaves) * (stage + 16u);
}

// Bytes of records staged per wave: what is left of the LDS after the tables.
uint32_t http_stage_bytes(const HttpHeader& h) {
  const size_t fixed = http_lds_bytes(h, 0) - kWaves * 16u;
  if (fixed + kWaves * (256u + 16u) > kHttpLdsBytes) return 0;
  size_t s = (kHttpLdsBytes - fixed) / kWaves - 16u;
  s &= ~size_t(15);
  return static_cast<uint32_t>(s > kMaxStage ? kMaxStage : s);
}

hipError_t launch_resident(ResidentBox* dbox, uint64_t first_seq, int kind, uint32_t* qhdr, hipStream_t stream) {
  return launch_kafka_resident(dbox, first_seq, kind, qhdr, stream);
}

hipError_t launch_http(const uint32_t* dprog, const HttpHeader& h, const uint8_t* arena, uint64_t arena_bytes,
                       const uint64_t* offs, uint64_t n, int32_t* verdicts, unsigned long long* hits,
                       hipStream_t stream, int num_cus, uint32_t flags, const DoneSignal* done) {
  if (n == 0) return hipSuccess;
  const uint32_t stage = http_stage_bytes(h);
  if (stage == 0) return hipErrorInvalidValue;
  const size_t lds = http_lds_bytes(h, stage);
  // kHttpWgPerCu resident workgroups per CU (1 by default); fewer for small
  // batches (>= 2 records per lane, two tiles per wave).
  uint64_t blocks = static_cast<uint64_t>(num_cus > 0 ? num_cus : 256) * kHttpWgPerCu;
  const uint64_t want = (n + 2 * kBlock - 1) / (2 * kBlock);
  if (want < blocks) blocks = want;
  const dim3 grid(static_cast<uint32_t>(blocks));
  const bool reg = h.n_dfas <= kRegDfas;
  if (flags & (L7M_FLAG_DIAG_WALK_ONLY | L7M_FLAG_DIAG_COPY_ONLY)) {  // diagnostic ablations
    // (register end codes only; no search automata, no slow-path queue)
    if (!reg || h.search || h.n_slow) return hipErrorInvalidValue;
    if (flags & L7M_FLAG_DIAG_COPY_ONLY)
      return launch_one<kNoHits, 8, 2>(grid, lds, stream, dprog, arena, arena_bytes, offs, n, verdicts, hits, stage);
    return launch_one<kNoHits, 8, 1>(grid, lds, stream, dprog, arena, arena_bytes, offs, n, verdicts, hits, stage);
  }
  const int mode = !hits ? kNoHits : (h.n_rules + 2 <= kMaxLdsCounters ? kLdsHits : kGlobalHits);
  // (kSliceHits) the workgroups' global counter slices, stream-ordered
  uint32_t* hslice = nullptr;
  if (kSliceHits && mode == kLdsHits) {
    const size_t bytes = static_cast<size_t>(grid.x) * ((h.n_rules + 2 + 63) & ~63u) * 4u;
    const hipError_t e = scratch_alloc_async(reinterpret_cast<void**>(&hslice), bytes, stream);
    if (e != hipSuccess) return e;
  }
  auto free_slice = [&](hipError_t e) {
    const hipError_t e2 = hslice ? hipFreeAsync(hslice, stream) : hipSuccess;
    return e != hipSuccess ? e : e2;
  };
  if (h.search) {
    // RE2-dialect programs (search automata, program.h kDfaSearch): their own
    // instantiation, end codes in a stream-ordered global scratch column per
    // thread (n_dfas words each)
    uint32_t* scratch = nullptr;
    const size_t bytes = static_cast<size_t>(h.n_dfas ? h.n_dfas : 1) * grid.x * kBlock * 4u;
    hipError_t e = scratch_alloc_async(reinterpret_cast<void**>(&scratch), bytes, stream);
    if (e != hipSuccess) return free_slice(e);
    const DoneSignal sig = done ? *done : DoneSignal{nullptr, nullptr, 0};
    if (mode == kNoHits) e = launch_one<kNoHits, -1>(grid, lds, stream, dprog, arena, arena_bytes, offs, n, verdicts,
                                                     hits, stage, scratch, nullptr, sig, hslice);
    else if (mode == kLdsHits) e = launch_one<kLdsHits, -1>(grid, lds, stream, dprog, arena, arena_bytes, offs, n,
                                                            verdicts, hits, stage, scratch, nullptr, sig, hslice);
    else e = launch_one<kGlobalHits, -1>(grid, lds, stream, dprog, arena, arena_bytes, offs, n, verdicts, hits, stage,
                                         scratch, nullptr, sig, hslice);
    const hipError_t e2 = hipFreeAsync(scratch, stream);
    return free_slice(e != hipSuccess ? e : e2);
  }
  // end codes in 4 or 8 registers, or in LDS columns
  const bool lit = (flags & kLaunchLiterals) != 0;
  const int R = h.n_dfas <= 4 ? 4 : reg ? 8 : 0;
  // programs with slow-path rules (program.h kCrSlow): the first pass queues
  // the requests they may decide, http_slow_kernel decides them; the queue
  // (count + up to n indices) and the executor scratch are stream-ordered
  uint32_t* slowq = nullptr;
  uint32_t* slowq2 = nullptr;
  uint32_t* vms = nullptr;
  uint32_t* vms2 = nullptr;
  uint32_t* work = nullptr;  // [0] tier-1, [64] tier-2 work counters
  const size_t qbytes = (4ull * (n + 1) + 255) & ~size_t(255);
  // tier 1: kSlowWavesPerCu waves per CU (fewer for small batches), tier 2: kSlowBlocks2 waves
  const uint64_t waves = (n + kSlowBlock - 1) / kSlowBlock;
  const uint64_t w1 = static_cast<uint64_t>(num_cus > 0 ? num_cus : 256) * kSlowWavesPerCu;
  const uint32_t blocks1 = static_cast<uint32_t>(waves < w1 ? waves : w1);
  const uint32_t blocks2 = static_cast<uint32_t>(waves < kSlowBlocks2 ? waves : kSlowBlocks2);
  void* buf = nullptr;  // the one stream-ordered allocation of the slow pass (freed by its base)
  if (h.n_slow) {
    const size_t v1 = static_cast<size_t>(blocks1) * kSlowBlock * kVmScratchWords * 4u;
    const size_t v2 = static_cast<size_t>(blocks2) * kSlowBlock * kVmScratchWords2 * 4u;
    hipError_t e = scratch_alloc_async(&buf, 512 + 2 * qbytes + v1 + v2, stream);
    if (e == hipSuccess) e = hipMemsetAsync(buf, 0, 512, stream);
    if (e == hipSuccess) e = hipMemsetAsync(static_cast<uint8_t*>(buf) + 512, 0, 4, stream);
    if (e == hipSuccess) e = hipMemsetAsync(static_cast<uint8_t*>(buf) + 512 + qbytes, 0, 4, stream);
    if (e != hipSuccess) {
      if (buf) (void)hipFreeAsync(buf, stream);
      return free_slice(e);
    }
    work = static_cast<uint32_t*>(buf);
    slowq = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(buf) + 512);
    slowq2 = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(buf) + 512 + qbytes);
    vms = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(buf) + 512 + 2 * qbytes);
    vms2 = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(buf) + 512 + 2 * qbytes + v1);
  }
  // the instantiation with the program's features (literal tables, forced
  // captures), each compiled in its own translation unit (l7m_http_feat.hip)
  const int feat = (lit ? kFeatLit : 0) | (h.lds_dcap != kNone ? kFeatDcap : 0);
  static decltype(&launch_http_main_f0) const mains[4] = {launch_http_main_f0, launch_http_main_f1,
                                                           launch_http_main_f2, launch_http_main_f3};
  static decltype(&launch_http_slow_f0) const slows[4] = {launch_http_slow_f0, launch_http_slow_f1,
                                                           launch_http_slow_f2, launch_http_slow_f3};
  // the completion signal only where this launch decides every request
  const DoneSignal sig = done && !h.n_slow ? *done : DoneSignal{nullptr, nullptr, 0};
  hipError_t e = mains[feat](mode, R, grid, lds, stream, dprog, arena, arena_bytes, offs, n, verdicts, hits, stage,
                             slowq, sig, hslice);
  if (h.n_slow) {
    for (int tier = 1; tier <= 2 && e == hipSuccess; ++tier)
      e = slows[feat](R, tier, h, tier == 1 ? blocks1 : blocks2, stream, dprog, arena, arena_bytes, offs, n, verdicts,
                      hits, slowq, slowq2, tier == 1 ? vms : vms2, work + (tier - 1) * 64);
    const hipError_t e2 = hipFreeAsync(buf, stream);
    if (e == hipSuccess) e = e2;
  }
  return free_slice(e);
}

}  // namespace l7m
