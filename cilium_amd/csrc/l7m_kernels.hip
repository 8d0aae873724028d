// l7m_kernels.hip — CDNA4 (gfx950) kernels of the batched L7 verdict path.
//
// HTTP: one lane per request (a wave evaluates 64 consecutive records of the
// arena).  Per request the lane streams the record's method / path /
// authority / header bytes through the per-field DFAs, one dependent table
// load per byte (`s = tab[s + cmap[b]]`, premultiplied rows, byte-class map
// staged in LDS), records the end set of every DFA in LDS, then resolves the
// first matching rule from the precomputed candidate lists (see
// http_compile.cc).  Reference semantics: NetworkPolicyMap::Allowed ->
// PortNetworkPolicyRule::Matches -> HttpNetworkPolicyRule::Matches ->
// ConfigUtility::matchHeaders (envoy/cilium_network_policy.h:68-237).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/l7match.h"
#include "l7m_device.h"
#include "program.h"

namespace l7m {

struct WalkDfa {
  const uint32_t* tab;
  const uint8_t* cmap;  // LDS
  uint32_t start, ncls;
};

// Stream `len` bytes at rec+pos through the DFA; returns the end-set id.
__device__ __forceinline__ uint32_t walk(const WalkDfa& d, const uint8_t* __restrict__ rec,
                                         uint32_t pos, uint32_t len) {
  uint32_t s = d.start;
  if (len) {
    const uint32_t* w32 = reinterpret_cast<const uint32_t*>(rec);
    uint32_t wi = pos >> 2;
    uint32_t word = __builtin_nontemporal_load(w32 + wi) >> (8 * (pos & 3));
    uint32_t avail = 4 - (pos & 3);
    for (uint32_t k = 0; k < len; ++k) {
      if (avail == 0) {
        ++wi;
        word = __builtin_nontemporal_load(w32 + wi);
        avail = 4;
      }
      uint32_t b = word & 0xffu;
      word >>= 8;
      --avail;
      s = d.tab[s + d.cmap[b]];
      if (s == 0) break;  // dead state: no pattern of this DFA can match
    }
  }
  return d.tab[s + d.ncls];
}

__device__ __forceinline__ WalkDfa load_dfa(const uint32_t* __restrict__ prog, const HttpHeader& h,
                                            const uint8_t* cmaps_lds, uint32_t k) {
  const DfaDesc* dd = reinterpret_cast<const DfaDesc*>(prog + h.off_dfas) + k;
  WalkDfa w;
  w.tab = prog + dd->table_off;
  w.cmap = cmaps_lds + 256u * dd->cmap_index;
  w.start = dd->start;
  w.ncls = dd->ncols - 1;
  return w;
}

__device__ __forceinline__ bool set_has(const uint32_t* __restrict__ pool, Span s, uint32_t p) {
  for (uint32_t j = 0; j < s.len; ++j) {
    uint32_t v = pool[s.off + j];
    if (v == p) return true;
    if (v > p) return false;  // sorted
  }
  return false;
}

// Per-wave aggregated counter increment: one atomic per distinct slot.
__device__ __forceinline__ void count_slot(unsigned long long* __restrict__ hits, uint32_t slot,
                                           bool active) {
  uint64_t todo = __ballot(active);
  const uint32_t lane = __lane_id();
  while (todo) {
    uint32_t leader = __builtin_ctzll(todo);
    uint32_t key = __shfl(slot, leader);
    uint64_t same = __ballot(active && slot == key) & todo;
    if (lane == leader) atomicAdd(hits + key, static_cast<unsigned long long>(__popcll(same)));
    todo &= ~same;
  }
}

template <bool kHits>
__global__ __launch_bounds__(256) void http_eval_kernel(const uint32_t* __restrict__ prog,
                                                        const uint8_t* __restrict__ arena,
                                                        uint64_t arena_bytes,
                                                        const uint64_t* __restrict__ offs,
                                                        uint64_t n, int32_t* __restrict__ verdicts,
                                                        unsigned long long* __restrict__ hits) {
  extern __shared__ __align__(16) uint8_t smem[];
  const HttpHeader h = *reinterpret_cast<const HttpHeader*>(prog);
  const uint32_t ndt = h.n_dfas + h.has_name_dfa;
  uint8_t* cmaps = smem;
  uint32_t* sids = reinterpret_cast<uint32_t*>(smem + 256u * ndt);
  {
    const uint32_t* g = prog + h.off_cmaps;
    uint32_t* l = reinterpret_cast<uint32_t*>(cmaps);
    for (uint32_t i = threadIdx.x; i < 64u * ndt; i += blockDim.x) l[i] = g[i];
  }
  __syncthreads();

  const uint32_t tid = threadIdx.x;
  const uint32_t bd = blockDim.x;
  const FieldDesc* fields = reinterpret_cast<const FieldDesc*>(prog + h.off_fields);
  const Span* sets = reinterpret_cast<const Span*>(prog + h.off_sets);
  const Span* cands = reinterpret_cast<const Span*>(prog + h.off_cands);
  const Span* rules = reinterpret_cast<const Span*>(prog + h.off_rules);
  const MatcherDesc* mds = reinterpret_cast<const MatcherDesc*>(prog + h.off_matchers);
  const DfaDesc* dds = reinterpret_cast<const DfaDesc*>(prog + h.off_dfas);
  const uint32_t* pool = prog + h.off_pool;
  const uint32_t* name_field = prog + h.off_name_field;
  const Span* remotes = reinterpret_cast<const Span*>(prog + h.off_remotes);

  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * bd;
  for (uint64_t r = static_cast<uint64_t>(blockIdx.x) * bd + tid; r < n; r += stride) {
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
    for (uint32_t d = 0; d < h.n_dfas; ++d) sids[d * bd + tid] = 0;

    uint32_t pos = L7M_HTTP_REC_FIXED + 4u * nhdr;
    auto eval_field = [&](uint32_t f, uint32_t p, uint32_t len) {
      const FieldDesc fd = fields[f];
      for (uint32_t k = 0; k < fd.ndfa; ++k) {
        WalkDfa wd = load_dfa(prog, h, cmaps, fd.dfa_first + k);
        sids[(fd.dfa_first + k) * bd + tid] = walk(wd, rec, p, len);
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
      WalkDfa nd = load_dfa(prog, h, cmaps, h.n_dfas);
      for (uint32_t j = 0; j < nhdr; ++j) {
        const uint32_t e = rw[5 + j];
        const uint32_t nl = e & 0xffffu, vl = e >> 16;
        const uint32_t sid = walk(nd, rec, pos, nl);
        const uint32_t f = sid ? name_field[sid] : kNone;
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
          const uint32_t sid = sids[m.dfa * bd + tid];
          if (sid == 0) return false;
          if (!set_has(pool, sets[dds[m.dfa].set_base + sid], m.pattern)) return false;
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
      const uint32_t sid = sids[d * bd + tid];
      if (sid) scan(cands[dds[d].set_base + sid]);
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

size_t http_lds_bytes(const HttpHeader& h, uint32_t block) {
  return 256u * (h.n_dfas + h.has_name_dfa) + static_cast<size_t>(h.n_dfas) * block * 4u;
}

hipError_t launch_http(const uint32_t* dprog, const HttpHeader& h, const uint8_t* arena,
                       uint64_t arena_bytes, const uint64_t* offs, uint64_t n, int32_t* verdicts,
                       unsigned long long* hits, hipStream_t stream, int num_cus) {
  if (n == 0) return hipSuccess;
  const uint32_t block = 256;
  uint64_t blocks = (n + block - 1) / block;
  uint64_t cap = static_cast<uint64_t>(num_cus > 0 ? num_cus : 256) * 8;
  if (blocks > cap) blocks = cap;
  size_t lds = http_lds_bytes(h, block);
  if (hits)
    hipLaunchKernelGGL(http_eval_kernel<true>, dim3(static_cast<uint32_t>(blocks)), dim3(block), lds,
                       stream, dprog, arena, arena_bytes, offs, n, verdicts, hits);
  else
    hipLaunchKernelGGL(http_eval_kernel<false>, dim3(static_cast<uint32_t>(blocks)), dim3(block), lds,
                       stream, dprog, arena, arena_bytes, offs, n, verdicts, hits);
  return hipGetLastError();
}

}  // namespace l7m
