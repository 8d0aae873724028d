// l7m_kernels.hip — CDNA4 (gfx950) kernel of the batched HTTP verdict path.
//
// One lane per request; a 512-thread workgroup is resident for many tiles of
// 512 consecutive records (grid-stride).  Per workgroup, once:
//   * the packed DFA slot tables that fit the LDS budget (the "LDS image",
//     dfa_pack.h) and the DFA descriptors are copied HBM -> LDS.
// Per request (lane):
//   * the record is streamed from HBM with 16-byte non-temporal loads (it is
//     read exactly once; non-temporal keeps the L2 for the rule tables);
//   * every referenced field (method / path / authority / header values whose
//     lower-cased name the header-name DFA recognises) is walked through its
//     DFA groups: ONE dependent 4-byte LDS read per input byte;
//   * the end codes select precomputed candidate rule lists; the first rule
//     (input order) whose remaining matchers hold is the verdict.
// Reference semantics: NetworkPolicyMap::Allowed -> PortNetworkPolicyRule::
// Matches -> HttpNetworkPolicyRule::Matches -> ConfigUtility::matchHeaders
// (envoy/cilium_network_policy.h:68-237).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/l7match.h"
#include "l7m_device.h"
#include "program.h"

namespace l7m {
namespace {

constexpr uint32_t kBlock = 512;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t sel4(const u32x4& v, uint32_t q) {
  uint32_t r = v.x;
  r = q == 1u ? v.y : r;
  r = q == 2u ? v.z : r;
  r = q == 3u ? v.w : r;
  return r;
}

// Walk `len` bytes at p through one packed DFA whose slot table is T (LDS or
// global).  Returns the end code: 0, a set id, or kLatchedBit | pattern.
template <bool kLds>
__device__ __forceinline__ uint32_t walk(const uint32_t* __restrict__ T, const DfaDesc& dd,
                                         const uint32_t* __restrict__ prog, const uint8_t* p, uint32_t len) {
  uint32_t desc = dd.start_desc;
  uint32_t last = kNone;
  if (len && desc) {
    const uint32_t region = dd.region;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const u32x4* cp = reinterpret_cast<const u32x4*>(a & ~uintptr_t(15));
    uint32_t o = static_cast<uint32_t>(a & 15u);
    u32x4 ch = __builtin_nontemporal_load(cp);
    uint32_t w = sel4(ch, o >> 2) >> (8u * (o & 3u));
    uint32_t base = desc >> 1;
    for (uint32_t k = 0;;) {
      const uint32_t slot = base + (w & 0xffu);
      const uint32_t e = T[slot];
      if (base < region) last = slot;
      desc = ((e & 0xffffu) == base) ? (e >> 16) : ((desc & 1u) ? desc : 0u);
      base = desc >> 1;
      if (++k == len || desc == 0u) break;
      ++o;
      w >>= 8;
      if ((o & 3u) == 0u) {
        if (o == 16u) {
          ++cp;
          ch = __builtin_nontemporal_load(cp);
          o = 0;
        }
        w = sel4(ch, o >> 2);
      }
    }
  }
  if (!desc) return 0;
  const uint32_t es = prog[dd.es_off + (desc >> 1)];
  if (es == kLatchedBit) return kLatchedBit | (last == kNone ? dd.start_latch : prog[dd.latch_off + last]);
  return es;
}

__device__ __forceinline__ uint32_t walk_any(const uint32_t* img, const DfaDesc& dd, const uint32_t* prog,
                                             const uint8_t* p, uint32_t len) {
  if (dd.lds_off != kNone) return walk<true>(img + dd.lds_off, dd, prog, p, len);
  return walk<false>(prog + dd.table_off, dd, prog, p, len);
}

__device__ __forceinline__ bool set_has(const uint32_t* __restrict__ pool, Span s, uint32_t p) {
  for (uint32_t j = 0; j < s.len; ++j) {
    const uint32_t v = pool[s.off + j];
    if (v == p) return true;
    if (v > p) return false;  // sorted
  }
  return false;
}

// Per-wave aggregated counter increment: one atomic per distinct slot.
__device__ __forceinline__ void count_slot(unsigned long long* __restrict__ hits, uint32_t slot, bool active) {
  uint64_t todo = __ballot(active);
  const uint32_t lane = __lane_id();
  while (todo) {
    const uint32_t leader = __builtin_ctzll(todo);
    const uint32_t key = __shfl(slot, leader);
    const uint64_t same = __ballot(active && slot == key) & todo;
    if (lane == leader) atomicAdd(hits + key, static_cast<unsigned long long>(__popcll(same)));
    todo &= ~same;
  }
}

template <bool kHits>
__global__ __launch_bounds__(kBlock) void http_eval_kernel(const uint32_t* __restrict__ prog,
                                                           const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                           const uint64_t* __restrict__ offs, uint64_t n,
                                                           int32_t* __restrict__ verdicts,
                                                           unsigned long long* __restrict__ hits) {
  extern __shared__ __align__(16) uint32_t smem[];
  const HttpHeader h = *reinterpret_cast<const HttpHeader*>(prog);
  const uint32_t ndt = h.n_dfas + h.has_name_dfa;
  uint32_t* img = smem;
  DfaDesc* dds = reinterpret_cast<DfaDesc*>(smem + h.lds_image_words);
  uint32_t* sids = smem + h.lds_image_words + 16u * ndt;
  const uint32_t tid = threadIdx.x;
  {
    const uint4* g = reinterpret_cast<const uint4*>(prog + h.lds_image_off);
    uint4* l = reinterpret_cast<uint4*>(img);
    for (uint32_t i = tid; i < h.lds_image_words / 4u; i += kBlock) l[i] = g[i];
    const uint4* gd = reinterpret_cast<const uint4*>(prog + h.off_dfas);
    uint4* ld = reinterpret_cast<uint4*>(dds);
    for (uint32_t i = tid; i < 4u * ndt; i += kBlock) ld[i] = gd[i];
  }
  __syncthreads();

  const FieldDesc* fields = reinterpret_cast<const FieldDesc*>(prog + h.off_fields);
  const Span* sets = reinterpret_cast<const Span*>(prog + h.off_sets);
  const Span* cands = reinterpret_cast<const Span*>(prog + h.off_cands);
  const Span* pcands = reinterpret_cast<const Span*>(prog + h.off_pcands);
  const Span* rules = reinterpret_cast<const Span*>(prog + h.off_rules);
  const MatcherDesc* mds = reinterpret_cast<const MatcherDesc*>(prog + h.off_matchers);
  const uint32_t* pool = prog + h.off_pool;
  const uint32_t* name_field = prog + h.off_name_field;
  const Span* remotes = reinterpret_cast<const Span*>(prog + h.off_remotes);

  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kBlock;
  for (uint64_t r = static_cast<uint64_t>(blockIdx.x) * kBlock + tid; r < n; r += stride) {
    const uint64_t off = offs[r];
    // Malformed record (outside the arena or inconsistent lengths): report
    // it instead of reading out of bounds.
    bool bad = (off & 3) || off + L7M_HTTP_REC_FIXED > arena_bytes;
    const uint8_t* rec = arena + (bad ? 0 : off);
    const uint32_t* rw = reinterpret_cast<const uint32_t*>(rec);
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0, w4 = 0;
    if (!bad) {
      w0 = rw[0];
      w1 = rw[1];
      w2 = rw[2];
      w3 = rw[3];
      w4 = rw[4];
    }
    const uint32_t flags = (w2 >> 16) & 0xffu;
    const uint32_t nhdr = w2 >> 24;
    const uint32_t mlen = w3 & 0xffffu, plen = w3 >> 16, alen = w4 & 0xffffu;
    if (!bad) {
      uint64_t need = L7M_HTTP_REC_FIXED + 4ull * nhdr + mlen + plen + alen;
      if (need > w0 || off + ((static_cast<uint64_t>(w0) + 3) & ~3ull) > arena_bytes) {
        bad = true;
      } else {
        for (uint32_t j = 0; j < nhdr; ++j) {
          const uint32_t e = rw[5 + j];
          need += (e & 0xffffu) + (e >> 16);
        }
        bad = need != w0;
      }
    }
    if (bad) {
      verdicts[r] = L7M_VERDICT_PARSE_ERROR;
      if (kHits) count_slot(hits, 1, true);
      continue;
    }
    uint64_t present = 0;
    for (uint32_t d = 0; d < h.n_dfas; ++d) sids[d * kBlock + tid] = 0;

    uint32_t pos = L7M_HTTP_REC_FIXED + 4u * nhdr;
    auto eval_field = [&](uint32_t f, uint32_t p, uint32_t len) {
      const FieldDesc fd = fields[f];
      for (uint32_t k = 0; k < fd.ndfa; ++k) {
        const uint32_t d = fd.dfa_first + k;
        sids[d * kBlock + tid] = walk_any(img, dds[d], prog, rec + p, len);
      }
    };
    if (flags & L7M_HTTP_F_METHOD) {
      present |= 1ull << kFieldMethod;
      eval_field(kFieldMethod, pos, mlen);
    }
    pos += mlen;
    if (flags & L7M_HTTP_F_PATH) {
      present |= 1ull << kFieldPath;
      eval_field(kFieldPath, pos, plen);
    }
    pos += plen;
    if (flags & L7M_HTTP_F_AUTHORITY) {
      present |= 1ull << kFieldAuthority;
      eval_field(kFieldAuthority, pos, alen);
    }
    pos += alen;
    if (h.has_name_dfa) {
      const DfaDesc& nd = dds[h.n_dfas];
      for (uint32_t j = 0; j < nhdr; ++j) {
        const uint32_t e = rw[5 + j];
        const uint32_t nl = e & 0xffffu, vl = e >> 16;
        const uint32_t code = walk_any(img, nd, prog, rec + pos, nl);
        uint32_t f = kNone;
        if (code & kLatchedBit) f = 3u + (code & ~kLatchedBit);
        else if (code) f = name_field[code];
        if (f != kNone && !((present >> f) & 1ull)) {  // first occurrence wins
          present |= 1ull << f;
          eval_field(f, pos + nl, vl);
        }
        pos += nl + vl;
      }
    }

    // First matching rule (smallest index) among the keyed candidates.
    uint32_t best = h.always_rule;
    const uint32_t remote = w1;
    auto verify = [&](uint32_t rid) -> bool {
      if (!h.any_remotes) {  // PortNetworkPolicyRule::Matches remote check (h:92-97)
        const Span rr = remotes[rid];
        if (rr.len) {
          uint32_t lo = 0, hi = rr.len;
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pool[rr.off + mid] < remote) lo = mid + 1;
            else hi = mid;
          }
          if (lo == rr.len || pool[rr.off + lo] != remote) return false;
        }
      }
      const Span rs = rules[rid];
      for (uint32_t j = 0; j < rs.len; ++j) {
        const MatcherDesc m = mds[rs.off + j];
        if (!((present >> m.field) & 1ull)) return false;
        if (m.kind == 0) {
          const uint32_t code = sids[m.dfa * kBlock + tid];
          if (code == 0) return false;
          if (code & kLatchedBit) {
            if ((code & ~kLatchedBit) != m.pattern) return false;
          } else if (!set_has(pool, sets[dds[m.dfa].set_base + code], m.pattern)) {
            return false;
          }
        }
      }
      return true;
    };
    auto scan = [&](Span c) {
      for (uint32_t j = 0; j < c.len; ++j) {
        const uint32_t rid = pool[c.off + j];
        if (rid >= best) break;
        if (verify(rid)) {
          best = rid;
          break;
        }
      }
    };
    for (uint32_t d = 0; d < h.n_dfas; ++d) {
      const uint32_t code = sids[d * kBlock + tid];
      if (code & kLatchedBit) scan(pcands[dds[d].pcand_base + (code & ~kLatchedBit)]);
      else if (code) scan(cands[dds[d].set_base + code]);
    }
    for (uint32_t f = 0; f < h.n_fields; ++f)
      if ((present >> f) & 1ull) scan(fields[f].presence);
    scan(h.zero_list);

    int32_t v;
    uint32_t slot;
    if (h.allow_no_l7) {
      v = L7M_VERDICT_ALLOW_NO_L7;
      slot = kNone;
    } else if (best == kNone) {
      v = L7M_VERDICT_DENY;
      slot = 0;
    } else {
      v = static_cast<int32_t>(best);
      slot = best + 2;
    }
    verdicts[r] = v;
    if (kHits) count_slot(hits, slot, slot != kNone);
  }
}

}  // namespace

size_t http_lds_bytes(const HttpHeader& h, uint32_t block) {
  (void)block;
  const size_t ndt = h.n_dfas + h.has_name_dfa;
  return 4u * (static_cast<size_t>(h.lds_image_words) + 16u * ndt + static_cast<size_t>(h.n_dfas) * kBlock);
}

hipError_t launch_http(const uint32_t* dprog, const HttpHeader& h, const uint8_t* arena, uint64_t arena_bytes,
                       const uint64_t* offs, uint64_t n, int32_t* verdicts, unsigned long long* hits,
                       hipStream_t stream, int num_cus) {
  if (n == 0) return hipSuccess;
  const size_t lds = http_lds_bytes(h, kBlock);
  // Workgroups stay resident for many tiles: size the grid to what fits.
  uint64_t per_cu = lds ? (160u * 1024u) / lds : 4;
  if (per_cu > 4) per_cu = 4;
  if (per_cu < 1) per_cu = 1;
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  const uint64_t cap = static_cast<uint64_t>(num_cus > 0 ? num_cus : 256) * per_cu;
  if (blocks > cap) blocks = cap;
  if (hits)
    hipLaunchKernelGGL(http_eval_kernel<true>, dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), lds, stream, dprog,
                       arena, arena_bytes, offs, n, verdicts, hits);
  else
    hipLaunchKernelGGL(http_eval_kernel<false>, dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), lds, stream, dprog,
                       arena, arena_bytes, offs, n, verdicts, hits);
  return hipGetLastError();
}

}  // namespace l7m
