// l7m_http_impl.h -- device code of the HTTP verdict kernels (design:
// l7m_kernels.hip).  Included by l7m_kernels.hip (search-dialect and
// diagnostic instantiations, the launcher) and by l7m_http_feat.hip, which
// instantiates the ECMAScript first-pass and slow-pass kernels of ONE
// feature set (kFeat) per translation unit, so they compile in parallel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/l7match.h"
#include "l7m_device.h"
#include "program.h"
#include "regex_vm.h"

namespace l7m {
namespace {

// geometry shared with the compiler (program.h)
constexpr uint32_t kWaves = kHttpWaves;
constexpr uint32_t kBlock = kHttpBlock;
constexpr uint32_t kMaxStage = kHttpMaxStage;  // bytes of records staged per wave and tile
constexpr uint32_t kCopyIters = (kMaxStage + 1023) / 1024;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#ifdef L7M_PROF
constexpr bool kProf = true;  // diagnostic build: wave timeline printed by two waves
#else
constexpr bool kProf = false;
#endif

// Explicit address-space loads where one expression picks between an LDS
// word and a program word: left generic, the compiler merges the two into a
// flat load of a selected pointer, and a flat load waits for vmcnt(0) AND
// lgkmcnt(0) -- i.e. for the next tile's bytes in flight.
typedef __attribute__((address_space(1))) const uint32_t* gptr_u32;
typedef __attribute__((address_space(3))) const uint32_t* lptr_u32;
__device__ __forceinline__ uint32_t gld(const uint32_t* p) { return *(gptr_u32)(p); }
__device__ __forceinline__ uint32_t lld(const uint32_t* p) { return *(lptr_u32)(p); }
// Byte i of a search automaton's class map: its LDS copy (lds: image byte
// address) or the program's (explicit address spaces: no flat load).
__device__ __forceinline__ uint32_t cmap_byte(uint32_t lds, const uint8_t* g, uint32_t i) {
  if (lds != kNone) return *reinterpret_cast<__attribute__((address_space(3))) const uint8_t*>(
                        static_cast<uintptr_t>(lds + i));
  return *(__attribute__((address_space(1))) const uint8_t*)(g + i);
}
// A program load whose wait is placed right here (in the branch that needs
// it): the verification phase runs after the next tile's bytes were
// requested, and a wait the compiler puts at a later join would be vmcnt(0)
// on every path through it, the common LDS-only one included.
__device__ __forceinline__ uint32_t gld_now(const uint32_t* p) {
  uint32_t v = gld(p);
  asm volatile("" : "+v"(v));
  return v;
}

// Where a record's bytes are read from.
struct LdsSrc {
  static constexpr bool kLds = true;
  const uint32_t* w;  // word 0 of the record in the wave's LDS stage
  __device__ __forceinline__ uint32_t word(uint32_t i) const { return w[i]; }
  __device__ __forceinline__ uint32_t byte(uint32_t i) const { return reinterpret_cast<const uint8_t*>(w)[i]; }
  // bytes [p, p + 4) from 4-byte-aligned reads and v_alignbyte: the byte
  // reads would be merged into a b64 read off its 8-byte alignment, which the
  // LDS replays (SQ_LDS_UNALIGNED_STALL 32 % of LDS-active cycles on config
  // 2; measured 3.516 vs 3.566 ms, profiles/r04/ab_round4.md)
  __device__ __forceinline__ uint32_t word_u(uint32_t p) const {
    const uint32_t* a = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(w) + (p & ~3u));
    return __builtin_amdgcn_alignbyte(a[1], a[0], p & 3u);
  }
};
struct GlbSrc {
  static constexpr bool kLds = false;
  const uint32_t* w;  // word 0 of the record in HBM
  __device__ __forceinline__ uint32_t word(uint32_t i) const { return __builtin_nontemporal_load(w + i); }
  __device__ __forceinline__ uint32_t byte(uint32_t i) const { return reinterpret_cast<const uint8_t*>(w)[i]; }
  __device__ __forceinline__ uint32_t word_u(uint32_t p) const {
    return byte(p) | byte(p + 1) << 8 | byte(p + 2) << 16 | byte(p + 3) << 24;
  }
};

// End code of a finished walk (final base, slot of the last transition taken
// from a multi-pattern state).
template <bool kLdsTab>
__device__ __forceinline__ uint32_t end_code(const uint32_t* __restrict__ img, const uint32_t* __restrict__ prog,
                                             const DfaDesc& dd, uint32_t base, uint32_t last) {
  if (!base) return 0;
  if (kLdsTab && dd.lds_es != kNone) {  // else: slot table in LDS, end codes in the program
    const uint16_t* I16 = reinterpret_cast<const uint16_t*>(img);
    const uint32_t es = I16[dd.lds_es + base];
    if (es != kEs16Latched) return es;
    return kLatchedBit | (last == kNone ? dd.start_latch : I16[dd.lds_latch + last]);
  }
  const uint32_t es = gld(prog + dd.es_off + base);
  if (es != kLatchedBit) return es;
  return kLatchedBit | (last == kNone ? dd.start_latch : gld(prog + dd.latch_off + last));
}

// Walk `len` bytes at byte `pos` of the record through one packed DFA
// (dfa_pack.h): per byte ONE dependent slot-table read.  The dead state is
// absorbing, so the exit test runs once per 8-byte block.
#define L7M_WALK_BYTES(STEP, DEAD)                                          \
  {                                                                         \
    for (; k + 8 <= len; k += 8) {  /* 8-byte blocks: half the loop */     \
      const uint32_t b0 = src.byte(pos + k), b1 = src.byte(pos + k + 1);    \
      const uint32_t b2 = src.byte(pos + k + 2), b3 = src.byte(pos + k + 3); \
      const uint32_t b4 = src.byte(pos + k + 4), b5 = src.byte(pos + k + 5); \
      const uint32_t b6 = src.byte(pos + k + 6), b7 = src.byte(pos + k + 7); \
      STEP(b0)                                                              \
      STEP(b1)                                                              \
      STEP(b2)                                                              \
      STEP(b3)                                                              \
      STEP(b4)                                                              \
      STEP(b5)                                                              \
      STEP(b6)                                                              \
      STEP(b7)                                                              \
      if (DEAD) break;                                                      \
    }                                                                       \
    if (k + 4 <= len && !(DEAD)) {  /* then at most one 4-byte block */    \
      const uint32_t b0 = src.byte(pos + k), b1 = src.byte(pos + k + 1);    \
      const uint32_t b2 = src.byte(pos + k + 2), b3 = src.byte(pos + k + 3); \
      STEP(b0)                                                              \
      STEP(b1)                                                              \
      STEP(b2)                                                              \
      STEP(b3)                                                              \
      k += 4;                                                               \
    }                                                                       \
    if (k < len && !(DEAD)) {  /* the last 1-3 bytes, no loop */           \
      STEP(src.byte(pos + k))                                               \
      if (k + 1 < len) {                                                    \
        STEP(src.byte(pos + k + 1))                                         \
        if (k + 2 < len) STEP(src.byte(pos + k + 2))                        \
      }                                                                     \
    }                                                                       \
  }

// HBM slot table: e = T[base + b]; base = (e & 0xff) == b ? e >> 8 : 0.
template <bool kLit, class Src>
__device__ __forceinline__ uint32_t walk_hbm(const uint32_t* __restrict__ img, const uint32_t* __restrict__ prog,
                                             const DfaDesc& dd, const Src& src, uint32_t pos, uint32_t len) {
  const uint32_t* __restrict__ T = prog + dd.table_off;
  const uint32_t region = dd.region;
  uint32_t base = dd.start_base;
  uint32_t last = kNone;
#define L7M_STEP(B)                                        \
  {                                                        \
    const uint32_t b_ = (B);                               \
    const uint32_t slot_ = base + b_;                      \
    const uint32_t e_ = T[slot_];                          \
    last = base < region ? slot_ : last;                   \
    base = (e_ & 0xffu) == b_ ? (e_ >> 8) : 0u;            \
  }
  uint32_t k = 0;
  if (!kLit || dd.lit_tab == kNone) {
    if (base) L7M_WALK_BYTES(L7M_STEP, !base)
    return end_code<false>(img, prog, dd, base, last);
  }
  // DFA with literal values (program.h lit_tab): 8-byte blocks until the walk
  // is latched on one pattern; a latched literal is then compared directly.
  bool lit_stop = false;
  if (base) {
    for (; k + 8 <= len; k += 8) {
      const uint32_t b0 = src.byte(pos + k), b1 = src.byte(pos + k + 1);
      const uint32_t b2 = src.byte(pos + k + 2), b3 = src.byte(pos + k + 3);
      const uint32_t b4 = src.byte(pos + k + 4), b5 = src.byte(pos + k + 5);
      const uint32_t b6 = src.byte(pos + k + 6), b7 = src.byte(pos + k + 7);
      L7M_STEP(b0)
      L7M_STEP(b1)
      L7M_STEP(b2)
      L7M_STEP(b3)
      L7M_STEP(b4)
      L7M_STEP(b5)
      L7M_STEP(b6)
      L7M_STEP(b7)
      if (!base) break;
      if (base >= region) {
        k += 8;
        lit_stop = true;
        break;
      }
    }
    if (base && !lit_stop) L7M_WALK_BYTES(L7M_STEP, !base)
  }
  if (lit_stop) {
    const uint32_t p = last == kNone ? dd.start_latch : gld(prog + dd.latch_off + last);
    const uint32_t lo = gld(prog + dd.lit_tab + 2 * p), ll = gld(prog + dd.lit_tab + 2 * p + 1);
    if (lo != kNone) {
      // bytes [0, k) followed the literal (the walk is latched on it): the
      // field matches iff it has the literal's length and the rest is equal
      if (ll != len) return 0;
      const uint8_t* L = reinterpret_cast<const uint8_t*>(prog + lo);
      uint32_t x = 0, i = k;
      for (; !x && i + 8 <= len; i += 8) {
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) x |= src.byte(pos + i + j) ^ L[i + j];
      }
      for (; !x && i < len; ++i) x |= src.byte(pos + i) ^ L[i];
      return x ? 0u : (kLatchedBit | p);
    }
    L7M_WALK_BYTES(L7M_STEP, !base)  // latched on a non-literal pattern: walk on
  }
#undef L7M_STEP
  return end_code<false>(img, prog, dd, base, last);
}

// A walk through an LDS slot table, re-encoded by the compiler for it
// (program.h kLdsRowShift): e = (image byte address of the next row << 16) |
// es8 << 8 | label, 0 for a dead transition (row 0: the zero dead row at the
// image start).  The label check of a step is folded into the address of the
// next read: with bp the byte the last read consumed,
//     a = row(e) + 4 b,  byte 3 of a = label(e) ^ bp;  e = lds[a]
// three VALU ops (SDWA byte / half-word selects, the xor writing byte 3 in
// place): a wrong label puts the address 16 MiB past the LDS, where a read
// returns 0, the dead row (measured: tools/lds_chain_bench.hip).  The walk is
// VALU-issue bound at 16 waves per CU (SQ_ACTIVE_INST_VALU ~60 % of the SIMD
// cycles), so VALU ops per byte are the cost: 3 here, 6 in the compare /
// select form.  `slast` (the slot of the last transition taken from a
// multi-pattern row, below lim) costs two more, so it is tracked only in the
// 8-byte blocks that start with a lane in the multi-pattern region: states
// never return there once they leave it (dfa_pack.h latching).
// The image must start at LDS address 0 (the kernels' only LDS array).
typedef __attribute__((address_space(3))) const uint32_t* lds_cptr;
__device__ __forceinline__ uint32_t lds_at(uint32_t byte_addr) {
  return *reinterpret_cast<lds_cptr>(static_cast<uintptr_t>(byte_addr));
}

// One step on byte SEL of W, the previous byte being PSEL of P.
#define L7M_OSTEP(W, SEL, P, PSEL, TRACK)                                                                      \
  {                                                                                                            \
    uint32_t t_;                                                                                               \
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" SEL        \
        : "=v"(t_)                                                                                             \
        : "v"(W));                                                                                             \
    asm("v_add_u32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"         \
        : "+v"(t_)                                                                                             \
        : "v"(e));                                                                                             \
    asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:" PSEL \
        : "+v"(t_)                                                                                             \
        : "v"(e), "v"(P));                                                                                     \
    if (TRACK) slast = (e >> kLdsRowShift) < lim ? t_ : slast;                                                 \
    e = lds_at(t_);                                                                                            \
  }

struct LdsChain {
  uint32_t e;      // the last entry read
  uint32_t pw;     // byte 3: the byte that read consumed
  uint32_t lim;    // byte address of the first latched row
  uint32_t t0;     // the table's image word offset
  uint32_t slast;  // slot byte address (kNone: none)
  __device__ __forceinline__ void init(const DfaDesc& dd) {
    t0 = dd.lds_table;
    lim = 4 * (dd.lds_table + dd.region);
    e = ((4 * (dd.lds_table + dd.start_base)) << kLdsRowShift) | (dd.start_es8 << 8);  // label 0
    pw = 0;
    slast = kNone;
  }
  __device__ __forceinline__ bool dead_now() const {
    return (e >> kLdsRowShift) == 0 || (e & 0xffu) != (pw >> 24);
  }
  template <class Src>
  __device__ __forceinline__ static uint32_t word_at(const Src& src, uint32_t p) {
    return src.word_u(p);
  }
  // continue the walk over bytes [k, len) of the field at pos
  template <class Src>
  __device__ __forceinline__ void run(const Src& src, uint32_t pos, uint32_t len, uint32_t k) {
    for (; k + 8 <= len; k += 8) {
      const uint32_t w0 = word_at(src, pos + k), w1 = word_at(src, pos + k + 4);
      if (__any((e >> kLdsRowShift) < lim)) {  // some lane may still leave the multi-pattern region
        L7M_OSTEP(w0, "BYTE_0", pw, "BYTE_3", true)
        L7M_OSTEP(w0, "BYTE_1", w0, "BYTE_0", true)
        L7M_OSTEP(w0, "BYTE_2", w0, "BYTE_1", true)
        L7M_OSTEP(w0, "BYTE_3", w0, "BYTE_2", true)
        L7M_OSTEP(w1, "BYTE_0", w0, "BYTE_3", true)
        L7M_OSTEP(w1, "BYTE_1", w1, "BYTE_0", true)
        L7M_OSTEP(w1, "BYTE_2", w1, "BYTE_1", true)
        L7M_OSTEP(w1, "BYTE_3", w1, "BYTE_2", true)
      } else {
        L7M_OSTEP(w0, "BYTE_0", pw, "BYTE_3", false)
        L7M_OSTEP(w0, "BYTE_1", w0, "BYTE_0", false)
        L7M_OSTEP(w0, "BYTE_2", w0, "BYTE_1", false)
        L7M_OSTEP(w0, "BYTE_3", w0, "BYTE_2", false)
        L7M_OSTEP(w1, "BYTE_0", w0, "BYTE_3", false)
        L7M_OSTEP(w1, "BYTE_1", w1, "BYTE_0", false)
        L7M_OSTEP(w1, "BYTE_2", w1, "BYTE_1", false)
        L7M_OSTEP(w1, "BYTE_3", w1, "BYTE_2", false)
      }
      pw = w1;
      if (dead_now()) return;
    }
    if (k + 4 <= len) {
      const uint32_t w0 = word_at(src, pos + k);
      L7M_OSTEP(w0, "BYTE_0", pw, "BYTE_3", true)
      L7M_OSTEP(w0, "BYTE_1", w0, "BYTE_0", true)
      L7M_OSTEP(w0, "BYTE_2", w0, "BYTE_1", true)
      L7M_OSTEP(w0, "BYTE_3", w0, "BYTE_2", true)
      pw = w0;
      k += 4;
    }
    for (; k < len; ++k) {
      const uint32_t b = src.byte(pos + k);
      L7M_OSTEP(b, "BYTE_0", pw, "BYTE_3", true)
      pw = b << 24;
    }
  }
  __device__ __forceinline__ uint32_t code(const uint32_t* __restrict__ img, const uint32_t* __restrict__ prog,
                                           const DfaDesc& dd) const {
    const bool ok = !dead_now();
    const uint32_t base = ok ? (e >> (kLdsRowShift + 2)) - t0 : 0u;
    const uint32_t last = slast == kNone ? kNone : ((slast & 0xffffffu) >> 2) - t0;
    if (dd.lds_es == kLdsEsInEntry) {  // the end code came with the last entry read
      if (!base) return 0;
      const uint32_t es = (e >> 8) & 0xffu;
      if (es != kEs8Latched) return es;
      const uint16_t* I16 = reinterpret_cast<const uint16_t*>(img);
      return kLatchedBit | (last == kNone ? dd.start_latch : I16[dd.lds_latch + last]);
    }
    return end_code<true>(img, prog, dd, base, last);
  }
};
#undef L7M_OSTEP

template <class Src>
__device__ __forceinline__ uint32_t walk_lds(const uint32_t* __restrict__ img, const uint32_t* __restrict__ prog,
                                             const DfaDesc& dd, const Src& src, uint32_t pos, uint32_t len) {
  LdsChain c;
  c.init(dd);
  if (dd.start_base) c.run(src, pos, len, 0);
  return c.code(img, prog, dd);
}

#undef L7M_WALK_BYTES

__device__ __forceinline__ bool set_has(const uint32_t* __restrict__ pool, Span s, uint32_t p) {
  for (uint32_t j = 0; j < s.len; ++j) {
    const uint32_t v = gld_now(pool + s.off + j);
    if (v == p) return true;
    if (v > p) return false;  // sorted
  }
  return false;
}

// Per-wave aggregated counter increment: one atomic per distinct slot.
// Must be called by every lane of the wave.
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

// Per-lane DFA end codes: in registers when the program has few value DFAs
// (static-index select chains, no scratch), else in an LDS column.
constexpr uint32_t kRegDfas = kHttpRegDfas;
template <int kReg>
struct Codes;
template <>
struct Codes<8> {
  // eight named registers: an array here is turned back into scratch memory
  uint32_t r0, r1, r2, r3, r4, r5, r6, r7;
  __device__ __forceinline__ void clear(uint32_t) { r0 = r1 = r2 = r3 = r4 = r5 = r6 = r7 = 0; }
  __device__ __forceinline__ void set(uint32_t d, uint32_t v) {
    r0 = d == 0 ? v : r0;
    r1 = d == 1 ? v : r1;
    r2 = d == 2 ? v : r2;
    r3 = d == 3 ? v : r3;
    r4 = d == 4 ? v : r4;
    r5 = d == 5 ? v : r5;
    r6 = d == 6 ? v : r6;
    r7 = d == 7 ? v : r7;
  }
  __device__ __forceinline__ uint32_t get(uint32_t d) const {
    const uint32_t a = d & 1 ? r1 : r0, b = d & 1 ? r3 : r2, e = d & 1 ? r5 : r4, f = d & 1 ? r7 : r6;
    const uint32_t lo = d & 2 ? b : a, hi = d & 2 ? f : e;
    return d & 4 ? hi : lo;
  }
};
template <>
struct Codes<4> {  // programs with <= 4 value DFAs: four registers
  uint32_t r0, r1, r2, r3;
  __device__ __forceinline__ void clear(uint32_t) { r0 = r1 = r2 = r3 = 0; }
  __device__ __forceinline__ void set(uint32_t d, uint32_t v) {
    r0 = d == 0 ? v : r0;
    r1 = d == 1 ? v : r1;
    r2 = d == 2 ? v : r2;
    r3 = d == 3 ? v : r3;
  }
  __device__ __forceinline__ uint32_t get(uint32_t d) const {
    const uint32_t a = d & 1 ? r1 : r0, b = d & 1 ? r3 : r2;
    return d & 2 ? b : a;
  }
};
template <>
struct Codes<0> {
  uint32_t* p;  // LDS, stride kBlock
  __device__ __forceinline__ void clear(uint32_t n) {
    for (uint32_t d = 0; d < n; ++d) p[d * kBlock] = 0;
  }
  __device__ __forceinline__ void set(uint32_t d, uint32_t v) { p[d * kBlock] = v; }
  __device__ __forceinline__ uint32_t get(uint32_t d) const { return p[d * kBlock]; }
};

// Programs with search automata (kReg = -1, RE2 dialect): one code word per
// value DFA, dozens of DFAs, kept in a global scratch column per thread
// (stride = the grid's threads); agent-scope loads and stores, so a later
// tile never reads a stale line of an earlier one.
// Search programs' end codes: the first kSearchRegCodes DFAs a record walks
// keep their codes in registers (the gram filter leaves a handful walked per
// record); more spill to a global scratch column per thread (stride = the
// grid's threads).  With <= 64 value DFAs a per-lane mask of the walked DFAs
// stands in for clearing the column.  (Round 4 kept every code in the
// column: config 2 RE2 spent ~40 % of a tile in verification on those L2
// round trips and the column evicted the search tables from L2.)
constexpr uint32_t kSearchRegCodes = 4;
template <>
struct Codes<-1> {
  uint32_t* p;
  uint32_t stride;
  uint64_t valid;
  bool masked;
  uint32_t nr;
  uint32_t rd[kSearchRegCodes], rv[kSearchRegCodes];
  __device__ __forceinline__ void clear(uint32_t n) {
    valid = 0;
    masked = n <= 64;
    nr = 0;
#pragma unroll
    for (uint32_t i = 0; i < kSearchRegCodes; ++i) rd[i] = kNone;
    if (!masked)
      for (uint32_t d = 0; d < n; ++d) __hip_atomic_store(p + d * stride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ __forceinline__ void set(uint32_t d, uint32_t v) {
    if (nr < kSearchRegCodes) {
#pragma unroll
      for (uint32_t i = 0; i < kSearchRegCodes; ++i) {
        rd[i] = nr == i ? d : rd[i];
        rv[i] = nr == i ? v : rv[i];
      }
      ++nr;
    } else {
      __hip_atomic_store(p + d * stride, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    valid |= d < 64 ? 1ull << d : 0ull;
  }
  // code |= bits (kDfaAlit groups collect their matched patterns one by one)
  __device__ __forceinline__ void orbits(uint32_t d, uint32_t bits) {
    bool f = false;
#pragma unroll
    for (uint32_t i = 0; i < kSearchRegCodes; ++i) {
      f |= rd[i] == d;
      rv[i] |= rd[i] == d ? bits : 0u;
    }
    if (f) return;
    if ((masked && !((valid >> d) & 1ull)) || nr < kSearchRegCodes) {
      set(d, bits | get(d));
      return;
    }
    const uint32_t v = __hip_atomic_load(p + d * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p + d * stride, v | bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    valid |= d < 64 ? 1ull << d : 0ull;
  }
  __device__ __forceinline__ uint32_t get(uint32_t d) const {
    if (masked && !((valid >> d) & 1ull)) return 0u;
    uint32_t r = 0;
    bool f = false;
#pragma unroll
    for (uint32_t i = 0; i < kSearchRegCodes; ++i) {
      r = rd[i] == d ? rv[i] : r;
      f |= rd[i] == d;
    }
    if (f) return r;
    uint32_t v = __hip_atomic_load(p + d * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("" : "+v"(v));
    return v;
  }
};

struct Ctx {
  const uint32_t* prog;
  const uint32_t* img;         // LDS image
  const DfaDesc* dds;          // LDS
  const FieldDesc* fields;     // LDS
  const uint32_t* name_field;  // LDS
  const Span* sets;            // HBM
  const uint32_t* pool;        // HBM
  const uint32_t* cr;          // HBM: check records
  const Span* remotes;         // HBM
};

// Search automaton (program.h kDfaSearch, RE2 dialect): the mask of the
// patterns matching some substring of the field -- per byte one dependent
// table read, and the mask of the patterns whose match ends there.
template <class Src>
__device__ __forceinline__ uint32_t walk_search(const Ctx& c, const DfaDesc& dd, const Src& src, uint32_t pos,
                                                uint32_t len) {
  const uint32_t* __restrict__ T = c.prog + dd.table_off;
  const uint8_t* __restrict__ cm = reinterpret_cast<const uint8_t*>(c.prog + dd.acc_cmap_off);
  const uint32_t cml = dd.lds_table != kNone ? 4u * dd.lds_table : kNone;  // class map in LDS (image byte address)
  const uint32_t* __restrict__ mid = c.prog + dd.acc_mid_off;
  const uint32_t ncls = dd.acc_ncls;
  uint32_t st = dd.start_base, acc = dd.start_es8;
  if (dd.lds_search != kNone) {  // small automaton: table and mid masks in LDS
    const uint32_t* LT = c.img + dd.lds_search;
    const uint32_t* LM = c.img + dd.lds_mid;
    for (uint32_t k = 0; k < len; ++k) {
      const uint32_t e = lld(LT + st * ncls + cmap_byte(cml, cm, src.byte(pos + k)));
      st = e & 0xffffffu;
      acc |= lld(LM + (e >> 24));
    }
    return acc | gld(c.prog + dd.es_off + st);
  }
  // mid masks in LDS when placed there (generic pointer: one flat read)
  const uint32_t* M = dd.lds_mid != kNone ? c.img + dd.lds_mid : mid;
  for (uint32_t k = 0; k < len; ++k) {
    const uint32_t e = gld(T + st * ncls + cmap_byte(cml, cm, src.byte(pos + k)));
    st = e & 0xffffffu;
    acc |= M[e >> 24];
  }
  return acc | gld(c.prog + dd.es_off + st);
}

// Up to four search automata (consecutive DFAs d0 .. d0 + m - 1 of one
// field) over the same bytes, interleaved: their table reads are independent,
// so m L2 round trips are in flight per byte instead of one (config 2 in the
// RE2 dialect walks ~32 automata per path).
// kL: every chain's table is in LDS (lds_search); else all are read from the
// program (LDS-resident tables have their program copy too).
constexpr uint32_t kSearchChains = 3;  // search automata walked at once per lane
template <bool kL, class Src>
__device__ __forceinline__ void walk_search4(const Ctx& c, uint32_t d0, uint32_t m, const Src& src, uint32_t pos,
                                             uint32_t len, uint32_t (&out)[kSearchChains]) {
  const uint32_t* T[kSearchChains];
  const uint8_t* cm[kSearchChains];
  const uint32_t* mid[kSearchChains];
  uint32_t ncls[kSearchChains], st[kSearchChains], acc[kSearchChains], cml[kSearchChains], lt[kSearchChains], lm[kSearchChains];
#pragma unroll
  for (uint32_t j = 0; j < kSearchChains; ++j) {
    const DfaDesc& dd = c.dds[d0 + (j < m ? j : 0u)];
    T[j] = c.prog + dd.table_off;
    cm[j] = reinterpret_cast<const uint8_t*>(c.prog + dd.acc_cmap_off);
    cml[j] = dd.lds_table != kNone ? 4u * dd.lds_table : kNone;
    mid[j] = dd.lds_mid != kNone ? c.img + dd.lds_mid : c.prog + dd.acc_mid_off;  // generic: LDS or program
    ncls[j] = dd.acc_ncls;
    st[j] = dd.start_base;
    acc[j] = dd.start_es8;
    lt[j] = dd.lds_search;  // kNone: table in the program (L2)
    lm[j] = dd.lds_mid;
  }
  for (uint32_t k = 0; k < len; ++k) {
    const uint32_t b = src.byte(pos + k);
#pragma unroll
    for (uint32_t j = 0; j < kSearchChains; ++j) {
      if (j < m) {
        const uint32_t ci = st[j] * ncls[j] + cmap_byte(cml[j], cm[j], b);
        const uint32_t e = kL ? lld(c.img + lt[j] + ci) : gld(T[j] + ci);
        st[j] = e & 0xffffffu;
        acc[j] |= kL ? lld(c.img + lm[j] + (e >> 24)) : mid[j][e >> 24];
      }
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < kSearchChains; ++j)
    out[j] = j < m ? acc[j] | gld(c.prog + c.dds[d0 + j].es_off + st[j]) : 0u;
}

// The same with a per-lane DFA per chain (the gram filter's selection):
// chain j walks DFA d[j] when j < m (m per lane).
template <bool kL, class Src>
__device__ __forceinline__ void walk_search4v(const Ctx& c, const uint32_t (&d)[kSearchChains], uint32_t m, const Src& src,
                                              uint32_t pos, uint32_t len, uint32_t (&out)[kSearchChains]) {
  const uint32_t* T[kSearchChains];
  const uint8_t* cm[kSearchChains];
  const uint32_t* mid[kSearchChains];
  uint32_t ncls[kSearchChains], st[kSearchChains], acc[kSearchChains], cml[kSearchChains], lt[kSearchChains], lm[kSearchChains];
#pragma unroll
  for (uint32_t j = 0; j < kSearchChains; ++j) {
    const DfaDesc& dd = c.dds[d[j < m ? j : 0u]];
    T[j] = c.prog + dd.table_off;
    cm[j] = reinterpret_cast<const uint8_t*>(c.prog + dd.acc_cmap_off);
    cml[j] = dd.lds_table != kNone ? 4u * dd.lds_table : kNone;
    mid[j] = dd.lds_mid != kNone ? c.img + dd.lds_mid : c.prog + dd.acc_mid_off;  // generic: LDS or program
    ncls[j] = dd.acc_ncls;
    st[j] = dd.start_base;
    acc[j] = dd.start_es8;
    lt[j] = dd.lds_search;  // kNone: table in the program (L2)
    lm[j] = dd.lds_mid;
  }
  for (uint32_t k = 0; k < len; ++k) {
    const uint32_t b = src.byte(pos + k);
#pragma unroll
    for (uint32_t j = 0; j < kSearchChains; ++j) {
      if (j < m) {
        const uint32_t ci = st[j] * ncls[j] + cmap_byte(cml[j], cm[j], b);
        const uint32_t e = kL ? lld(c.img + lt[j] + ci) : gld(T[j] + ci);
        st[j] = e & 0xffffffu;
        acc[j] |= kL ? lld(c.img + lm[j] + (e >> 24)) : mid[j][e >> 24];
      }
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < kSearchChains; ++j) out[j] = j < m ? acc[j] | gld(c.prog + c.dds[d[j]].es_off + st[j]) : 0u;
}

// RE2-dialect gram filter (program.h FieldDesc::gram_tab): bit j % 32 of the
// result = the field's search group j may match.  Every 4-byte window of the
// value is one independent probe of a 2-entry LDS bucket (no dependent chain).
template <class Src>
__device__ __forceinline__ uint32_t gram_select(const Ctx& c, const FieldDesc& fd, const Src& src, uint32_t pos,
                                                uint32_t len) {
  uint32_t m = fd.always;
  if (len < 4) return m;
  const u32x4* tab = reinterpret_cast<const u32x4*>(c.img + fd.gram_tab);
  const uint32_t gm = fd.gram_mask, end = pos + len - 3;  // grams start in [pos, end)
  auto probe = [&](uint32_t g, bool on) {
    const u32x4 e = tab[on ? gram_bucket(g) & gm : 0u];
    m |= on ? ((e.x == g ? e.y : 0u) | (e.z == g ? e.w : 0u)) : 0u;
  };
  if constexpr (Src::kLds) {
    uint32_t q = pos & ~3u;
    uint32_t w0 = src.word(q >> 2);
    for (; q < end; q += 4) {
      const uint32_t w1 = src.word((q >> 2) + 1);
#pragma unroll
      for (uint32_t sft = 0; sft < 4; ++sft)
        probe(__builtin_amdgcn_alignbyte(w1, w0, sft), q + sft >= pos && q + sft < end);
      w0 = w1;
    }
  } else {
    for (uint32_t q = pos; q < end; ++q) probe(src.word_u(q), true);
  }
  return m;
}

template <bool kLit, bool kSearch, class Src>
__device__ __forceinline__ uint32_t walk_dfa(const Ctx& c, uint32_t d, const Src& src, uint32_t pos, uint32_t len);
template <bool kSearch>
__device__ __forceinline__ bool code_has(const Ctx& c, uint32_t d, uint32_t code, uint32_t p);

// Literal-anchored RE2 patterns of a field (program.h FieldDesc::alit_*):
// every value position q whose 4-byte gram hits an entry of the LDS bucket
// table names a pattern L R whose table gram sits at offset k of L; L is
// compared at q - k (program memory, word-wise) and the residual automaton
// is walked from the end of L; a match sets the pattern's bit in its kDfaAlit
// group's code.  Positions are probed from aligned words (one LDS read per
// four positions plus the bucket reads, all independent); only the lanes
// with a hit run the compare and the residual walk.
template <int kReg, class Src>
__device__ __forceinline__ void alit_scan(const Ctx& c, const FieldDesc& fd, const Src& src, uint32_t pos,
                                          uint32_t len, Codes<kReg>& codes) {
  if (len < 4) return;
  const u32x4* tab = reinterpret_cast<const u32x4*>(c.img + fd.alit_tab);
  const uint32_t am = fd.alit_mask, end = pos + len - 3;  // grams start in [pos, end)
  const uint32_t ngran = fd.alit_granules;
  auto candidate = [&](uint32_t rec, uint32_t q) {
    // rec comes from a bucket entry whose hit bit required it non-zero, so it
    // is a compiled AlitRec granule; the bound keeps any other value (an
    // ablated or corrupted scan, r5g's `skip` variant) from forming a pointer
    // outside the records
    if (rec >= ngran) return;
    // the AlitRec in LDS or the program (generic pointer): its header and the
    // first 16 literal bytes in one 32-byte read
    const u32x4* rp = reinterpret_cast<const u32x4*>(fd.alit_lds ? c.img : c.prog) + (fd.alit_pats >> 2) + rec;
    const u32x4 a0 = rp[0], a1 = rp[1];
    const uint32_t ln = a0.x & 0xffffu, k = a0.x >> 16;
    if (q < pos + k) return;
    const uint32_t s = q - k;  // candidate start (record byte offset)
    if (s + ln > pos + len) return;
    bool eq = true;
    for (uint32_t i = 0; eq && i < ln; i += 4) {
      const uint32_t j = i >> 2;
      const uint32_t lw = j == 0 ? a1.x : j == 1 ? a1.y : j == 2 ? a1.z : j == 3 ? a1.w
                                                                              : reinterpret_cast<const uint32_t*>(rp + 1)[j];
      const uint32_t sw = src.word_u(s + i);
      const uint32_t rem = ln - i;
      const uint32_t m = rem >= 4 ? 0xffffffffu : (1u << (8 * rem)) - 1u;
      eq = ((lw ^ sw) & m) == 0;
    }
    if (!eq) return;
    if (a0.z != kNone) {
      const uint32_t rc = walk_dfa<false, false>(c, fd.resid_dfa, src, s + ln, pos + len - (s + ln));
      if (!code_has<false>(c, fd.resid_dfa, rc, a0.z)) return;
    }
    codes.orbits(a0.y >> 8, 1u << (a0.y & 31u));
    // the pattern's candidate entry is read by verification: start its L2
    // round trip now (as the packed walks' touch does)
    const DfaDesc& gd = c.dds[a0.y >> 8];
    if (gd.lds_ct == kNone) {
      uint32_t t = gld(c.prog + gd.ct_off + 16u * (a0.y & 31u));
      asm volatile("" ::"v"(t));
    }
  };
  // Windows of 32 positions.  The probes of a window only set hit bits, one
  // per position whose gram hits its bucket -- no candidate work inside the
  // probe loop, whose iterations differ per lane --; then each hit re-reads
  // its bucket and runs the literal compare / residual walk of each matching
  // entry from one call site.  The optional prefilter (program.h
  // L7M_ALIT_BLOOM_BITS: one bit of a 2^bits map below the bucket table per
  // position, a dword read and a bit-field extract instead of the 16-byte
  // bucket read and two compares) measured slower on config 2 (round 6,
  // profiles/r06/ab_re2_prefilter_*: 2^14 bits 13.4 ms, 2^12 14.3 ms, off
  // 12.9 ms): its LDS costs record stage, and its false positives re-read
  // buckets, so it is off by default.
  const uint32_t* bloom = c.img + fd.alit_tab - kAlitBloomWords;
  auto bloom_hit = [&](uint32_t g) -> uint32_t {
    const uint32_t b = alit_bloom_bit(gram_bucket(g));
    return __builtin_amdgcn_ubfe(lld(bloom + (b >> 5)), b & 31u, 1);
  };
  // without the prefilter (kAlitBloomBits 0, round 5): the bucket itself
  auto bucket_hit = [&](uint32_t g) -> uint32_t {
    const u32x4 e = tab[gram_bucket(g) & am];
    return (e.y && e.x == g) || (e.w && e.z == g) ? 1u : 0u;
  };
  auto probe = [&](uint32_t g) -> uint32_t { return kAlitBloomBits ? bloom_hit(g) : bucket_hit(g); };
  for (uint32_t base = pos & ~3u; base < end; base += 32) {
    uint32_t hm = 0;
    if constexpr (Src::kLds) {
      uint32_t w0 = src.word(base >> 2);
      for (uint32_t i = 0; i < 8 && base + 4 * i < end; ++i) {
        const uint32_t w1 = src.word((base >> 2) + i + 1);
#pragma unroll
        for (uint32_t sft = 0; sft < 4; ++sft) {
          const uint32_t q = base + 4 * i + sft;
          const uint32_t h = probe(__builtin_amdgcn_alignbyte(w1, w0, sft));
          hm |= (q >= pos && q < end ? h : 0u) << (4 * i + sft);
        }
        w0 = w1;
      }
    } else {
      for (uint32_t i = 0; i < 32 && base + i < end; ++i) {
        const uint32_t q = base + i;
        if (q < pos) continue;
        hm |= probe(src.word_u(q)) << i;
      }
    }
    while (hm) {
      const uint32_t j = static_cast<uint32_t>(__builtin_ctz(hm));
      hm &= hm - 1;
      const uint32_t q = base + j, g = src.word_u(q);
      const u32x4 e = tab[gram_bucket(g) & am];
      uint32_t m2 = (e.y && e.x == g ? 1u : 0u) | (e.w && e.z == g ? 2u : 0u);
      while (m2) {
        const uint32_t k = static_cast<uint32_t>(__builtin_ctz(m2));
        m2 &= m2 - 1;
        candidate((k ? e.w : e.y) - 1, q);
      }
    }
  }
}

template <bool kLit, bool kSearch, class Src>
__device__ __forceinline__ uint32_t walk_dfa(const Ctx& c, uint32_t d, const Src& src, uint32_t pos, uint32_t len) {
  const DfaDesc& dd = c.dds[d];
  if (kSearch && dd.kind == kDfaSearch) return walk_search(c, dd, src, pos, len);
  if (dd.lds_table != kNone) return walk_lds(c.img, c.prog, dd, src, pos, len);
  return walk_hbm<kLit>(c.img, c.prog, dd, src, pos, len);
}

// Field id of the header name at byte `pos` (length len) of the record, via
// the LDS header-name table (program.h): the name's words are read aligned
// and hashed word-wise, one slot probe, one word-wise compare.  kNone if no
// rule references the name.
template <class Src>
__device__ __forceinline__ uint32_t name_field_of(const Ctx& c, const HttpHeader& h, const Src& src, uint32_t pos,
                                                  uint32_t len) {
  constexpr uint32_t kW = kNameHashMinWords;
  const uint32_t sh = pos & 3u, w0 = pos >> 2;
  uint32_t w[kW + 1], x[kW];
#pragma unroll
  for (uint32_t k = 0; k <= kW; ++k) w[k] = (Src::kLds || 4 * k < sh + len) ? src.word(w0 + k) : 0u;
  uint32_t hh = 0;
#pragma unroll
  for (uint32_t k = 0; k < kW; ++k) {
    x[k] = 0;
    if (__any(4 * k < len)) {  // words past every lane's name are skipped
      const uint32_t v = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
      const int32_t rem = static_cast<int32_t>(len) - static_cast<int32_t>(4 * k);
      x[k] = rem >= 4 ? v : rem <= 0 ? 0u : v & ((1u << (8 * rem)) - 1u);
      if (rem > 0) hh = name_hash_step(hh, x[k]);
    }
  }
  for (uint32_t i = 4 * kW; i < len; i += 4) {  // names longer than 24 bytes
    uint32_t y = 0;
    for (uint32_t b = 0; b < 4 && i + b < len; ++b) y |= src.byte(pos + i + b) << (8 * b);
    hh = name_hash_step(hh, y);
  }
  hh = name_hash_final(hh, len);
  const uint32_t* tab = c.img + h.lds_name_tab;
  for (uint32_t at = hh & h.name_tab_mask;; at = (at + 1) & h.name_tab_mask) {
    const u32x4 sl = reinterpret_cast<const u32x4*>(tab)[at];
    if (sl.x == 0) return kNone;
    if (sl.x != hh || sl.y != len) continue;
    const uint32_t* nw = c.img + sl.w;
    bool eq = true;
#pragma unroll
    for (uint32_t k = 0; k < kW; ++k)
      if (4 * k < len) eq &= x[k] == nw[k];
    for (uint32_t i = 4 * kW; eq && i < len; ++i)
      eq = src.byte(pos + i) == reinterpret_cast<const uint8_t*>(nw)[i];
    if (eq) return sl.z;
  }
}

// Does end code `code` of DFA d contain pattern p?
template <bool kSearch>
__device__ __forceinline__ bool code_has(const Ctx& c, uint32_t d, uint32_t code, uint32_t p) {
  if (code == 0) return false;
  const DfaDesc& dd = c.dds[d];
  if (kSearch && dd.kind != kDfaPacked) return ((code >> p) & 1u) != 0;  // code = matched-pattern mask
  if (code & kLatchedBit) return (code & ~kLatchedBit) == p;
  if (dd.lds_mask != kNone) {
    const uint32_t* m = c.img + dd.lds_mask + 2u * code;
    return ((p < 32 ? m[0] >> p : m[1] >> (p - 32)) & 1u) != 0;
  }
  const uint32_t* sp = reinterpret_cast<const uint32_t*>(c.sets + dd.set_base + code);
  return set_has(c.pool, Span{gld_now(sp), gld_now(sp + 1)}, p);
}

// (policy, direction, port) -> entry | kEntHaveHttp, or kNone (program.h).
__device__ __forceinline__ uint32_t ent_lookup(const Ctx& c, const HttpHeader& h, uint32_t key) {
  const bool lds = h.lds_ent_tab != kNone;
  const uint32_t* tab = lds ? c.img + h.lds_ent_tab : c.prog + h.ent_tab_off;
  for (uint32_t at = ent_hash(key) & h.ent_mask;; at = (at + 1) & h.ent_mask) {
    const uint32_t k = lds ? lld(tab + 2 * at) : gld(tab + 2 * at);
    if (k == 0) return kNone;
    if (k == key + 1) return lds ? lld(tab + 2 * at + 1) : gld(tab + 2 * at + 1);
  }
}

constexpr uint32_t kMinStagedTake = 32;

// Diagnostic timeline (L7M_PROF builds, kProf): per-lane cycle accumulators
// per evaluation phase (s_memtime), LDS-staged records only; prof[0] = last
// timestamp.  Without kProf the accumulators are dead stores and vanish.
template <bool kLds>
__device__ __forceinline__ void hprof(uint64_t (&prof)[8], int i) {
  if constexpr (kProf && kLds) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    prof[i] += t - prof[0];
    prof[0] = t;
  }
}
#define HPROF(i) hprof<Src::kLds>(prof, i)

// Forced-capture back-reference pattern (program.h DcapSpec, regex_ecma.h
// DcapForm) on the field value [p, p + len): P1, the maximal class run, L2,
// the run again, R's automaton over the rest -- exactly regex_match's answer.
template <bool kLit, class Src>
__device__ __forceinline__ bool dcap_holds(const Ctx& c, const DcapSpec& sp, const Src& src, uint32_t p, uint32_t len) {
  const uint32_t l1 = sp.lens & 0xffffu, l2 = sp.lens >> 16;
  if (len < l1 + l2) return false;
  const uint8_t* P1 = reinterpret_cast<const uint8_t*>(c.img + sp.p1);
  const uint8_t* L2 = reinterpret_cast<const uint8_t*>(c.img + sp.l2);
  for (uint32_t i = 0; i < l1; ++i)
    if (src.byte(p + i) != P1[i]) return false;
  uint32_t e = l1;
  while (e < len) {
    const uint32_t b = src.byte(p + e);
    if (!((sp.cls[b >> 5] >> (b & 31u)) & 1u)) break;
    ++e;
  }
  const uint32_t r = e - l1;
  if (r < sp.min || r > sp.max) return false;  // max kNone: unbounded
  if (static_cast<uint64_t>(e) + l2 + r > len) return false;
  for (uint32_t i = 0; i < l2; ++i)
    if (src.byte(p + e + i) != L2[i]) return false;
  for (uint32_t i = 0; i < r; ++i)
    if (src.byte(p + e + l2 + i) != src.byte(p + l1 + i)) return false;
  const uint32_t t = e + l2 + r;
  if (sp.rdfa == kNone) return t == len;
  const uint32_t code = walk_dfa<kLit, false>(c, sp.rdfa, src, p + t, len - t);
  return code_has<false>(c, sp.rdfa, code, 0);
}

// What the walk phase of a record hands to its verification phase.
template <int kReg>
struct WalkOut {
  Codes<kReg> codes;  // end code per value DFA
  uint64_t present;   // fields present in the request
  uint32_t ex, e0;    // port entries whose rules may decide (exact port, port 0)
  uint32_t remote;    // the request's remote identity
  uint32_t pf_t;      // the candidate-entry touch (kept live until verification)
  uint32_t dcap;      // bit k: forced-capture pattern k holds on its field (program.h DcapSpec)
  bool h0;            // the port-0 entry has HTTP rules
};
constexpr int32_t kNeedVerify = INT32_MIN;
// Instantiation features of the HTTP kernels (template parameter kFeat):
// kFeatLit: the program has literal tables (DfaDesc::lit_tab) for HBM-walked
// DFAs; kFeatDcap: it has forced-capture back-reference patterns (program.h
// DcapSpec).  Programs without them run the plain instantiation, whose code
// and register allocation neither feature touches.
constexpr int kFeatLit = 1, kFeatDcap = 2;
// First pass: the request's smallest candidate may be a slow-path rule
// (kCrSlow): it is queued for http_slow_kernel, which decides it exactly.
constexpr int32_t kDeferred = INT32_MIN + 1;
constexpr int32_t kDeferred2 = INT32_MIN + 2;  // slow pass, tier 1 -> tier 2 (regex_vm.h)

// Where field f's value lies in a record (slow pass): the pseudo headers from
// the fixed part, other fields as the first header whose name maps to f (the
// walk phase's header-name lookup).  false if absent.
template <class Src>
__device__ bool field_at(const Ctx& c, const HttpHeader& h, const Src& src, uint32_t f, uint32_t* pos,
                         uint32_t* len) {
  const uint32_t w2 = src.word(2), w3 = src.word(3), w4 = src.word(4);
  const uint32_t flags = (w2 >> 16) & 0xffu, nhdr = w2 >> 24;
  const uint32_t mlen = w3 & 0xffffu, plen = w3 >> 16, alen = w4 & 0xffffu;
  uint32_t p = L7M_HTTP_REC_FIXED + 4u * nhdr;
  if (f < 3) {
    if (!(flags & (f == 0 ? L7M_HTTP_F_METHOD : f == 1 ? L7M_HTTP_F_PATH : L7M_HTTP_F_AUTHORITY))) return false;
    *pos = p + (f >= 1 ? mlen : 0u) + (f == 2 ? plen : 0u);
    *len = f == 0 ? mlen : f == 1 ? plen : alen;
    return true;
  }
  p += mlen + plen + alen;
  for (uint32_t j = 0; j < nhdr; ++j) {
    const uint32_t e = src.word(5 + j), nl = e & 0xffffu, vl = e >> 16;
    uint32_t g = kNone;
    if (h.lds_name_tab != kNone) {
      g = name_field_of(c, h, src, p, nl);
    } else {
      const uint32_t code = walk_dfa<false, false>(c, h.n_dfas, src, p, nl);
      if (code & kLatchedBit) g = 3u + (code & ~kLatchedBit);
      else if (code) g = c.name_field[code];
    }
    if (g == f) {
      *pos = p + nl;
      *len = vl;
      return true;
    }
    p += nl + vl;
  }
  return false;
}

// Walk phase of one record whose first `limit` bytes are readable: record
// validation, port-entry selection and every DFA walk.  Returns the verdict
// when it is decided without rules, else kNeedVerify with `o` filled in.
// kAblate (diagnostic builds selected by L7M_FLAG_DIAG_*; verdicts invalid):
// 1 = stop after the DFA walks, 2 = stop after record validation.
template <int kReg, int kAblate, int kFeat, class Src>
__device__ __forceinline__ int32_t eval_walk(const Ctx& c, const HttpHeader& h, const Src& src, uint64_t limit,
                                             WalkOut<kReg>& o, uint64_t (&prof)[8]) {
  if constexpr (kProf && Src::kLds) prof[0] = __builtin_amdgcn_s_memtime();
  constexpr bool kLit = (kFeat & kFeatLit) != 0, kDcap = (kFeat & kFeatDcap) != 0;
  Codes<kReg>& codes = o.codes;
  if (limit < L7M_HTTP_REC_FIXED) return L7M_VERDICT_PARSE_ERROR;
  const uint32_t w0 = src.word(0), w1 = src.word(1), w2 = src.word(2), w3 = src.word(3), w4 = src.word(4);
  const uint32_t flags = (w2 >> 16) & 0xffu;
  const uint32_t nhdr = w2 >> 24;
  const uint32_t mlen = w3 & 0xffffu, plen = w3 >> 16, alen = w4 & 0xffffu;
  uint64_t need = L7M_HTTP_REC_FIXED + 4ull * nhdr + mlen + plen + alen;
  if (need > w0 || ((static_cast<uint64_t>(w0) + 3) & ~3ull) > limit) return L7M_VERDICT_PARSE_ERROR;
  for (uint32_t j = 0; j < nhdr; ++j) {
    const uint32_t e = src.word(5 + j);
    need += (e & 0xffffu) + (e >> 16);
  }
  if (need != w0) return L7M_VERDICT_PARSE_ERROR;

  if constexpr (kAblate == 2) return static_cast<int32_t>(w0 & 7u);

  // Port entry selection, PortNetworkPolicy::Matches (cilium_network_policy.h
  // :169-192) under NetworkPolicyMap::Allowed (h:223-237): the request's
  // endpoint policy and direction select the exact-port entry `ex` and the
  // port-0 entry `e0`; exact-port rules precede port-0 rules in the index
  // order, so the smallest matching index is Envoy's first true.
  uint32_t ex = 0, e0 = 0;
  bool h0 = true;
  {
    const uint32_t pol = w4 >> 16;
    if (h.single_entry) {
      if (pol != 0) return L7M_VERDICT_DENY;  // unknown endpoint policy (h:231-235)
      if (h.allow_no_l7) return L7M_VERDICT_ALLOW_NO_L7;
    } else {
      if (pol >= h.n_policies) return L7M_VERDICT_DENY;
      const uint32_t key0 = ent_key(pol, flags & L7M_HTTP_F_INGRESS, 0);
      const uint32_t vx = (w2 & 0xffffu) ? ent_lookup(c, h, key0 | (w2 & 0xffffu)) : kNone;
      const uint32_t v0 = ent_lookup(c, h, key0);
      if (vx == kNone && v0 == kNone) return L7M_VERDICT_ALLOW_NO_PORT_POLICY;
      const uint32_t first = vx != kNone ? vx : v0;
      if (!(first & kEntHaveHttp)) return L7M_VERDICT_ALLOW_NO_L7;  // h:129-135
      ex = first & ~kEntHaveHttp;
      e0 = (vx != kNone && v0 != kNone) ? (v0 & ~kEntHaveHttp) : ex;
      h0 = (vx != kNone && v0 != kNone) ? (v0 & kEntHaveHttp) != 0 : true;
    }
  }
  HPROF(1);
  uint64_t present = 0;
  codes.clear(h.n_dfas);
  // Walk jobs, one loop so that the walk code exists once in the kernel
  // (instruction-cache footprint): 0 method, 1 path, 2 authority, then the
  // values of headers whose name a rule references (first occurrence).  The
  // job index is wave-uniform; for the header jobs each lane first moves its
  // cursor (hj, hp) past headers whose name length no rule uses, so a wave
  // runs one job per referenced header, not one per header.
  uint32_t pos = L7M_HTTP_REC_FIXED + 4u * nhdr;
  uint32_t hj = 0, hp = pos + mlen + plen + alen;
  // DFAs with candidate entries (a uniform mask when n_dfas <= 64)
  const bool masked = h.n_dfas <= 64;
  const uint64_t cand_all = masked ? ((static_cast<uint64_t>(h.cand_dfas_hi) << 32) | h.cand_dfas_lo) : 0;
  // The candidate entry (program memory) of the first walk that selects one
  // is touched (one dword load) as soon as that walk ends, so its L2 round
  // trip overlaps the remaining walks and verification reads the entry from
  // the CU's L1 (the walks in between touch no global memory).
  bool touched = false;
  uint32_t pf_t = 0;
  auto touch = [&](uint32_t d, uint32_t code) {
    if (!touched && code && ((cand_all >> d) & 1ull)) {
      const DfaDesc& dd = c.dds[d];
      if (dd.lds_ct == kNone && !(kReg < 0 && dd.kind != kDfaPacked)) {
        const uint32_t idx = (code & kLatchedBit) ? dd.nsets + (code & ~kLatchedBit) : code;
        pf_t = c.prog[dd.ct_off + 16u * idx];
        touched = true;
      }
    }
  };
  uint32_t dcap = 0;
  const DcapSpec* dspec = reinterpret_cast<const DcapSpec*>(c.img + (kDcap ? h.lds_dcap : 0u));
  for (uint32_t job = 0;; ++job) {
    HPROF(4);  // (diagnostic build) what followed the previous job's walks
    uint32_t f = kNone, p = pos, len = 0;
    if (job < 3) {
      len = job == 0 ? mlen : job == 1 ? plen : alen;
      if (flags & (job == 0 ? L7M_HTTP_F_METHOD : job == 1 ? L7M_HTTP_F_PATH : L7M_HTTP_F_AUTHORITY)) f = job;
      pos += len;
    } else {
      if (!h.has_name_dfa) break;
      uint32_t e = 0;
      for (; hj < nhdr; ++hj) {
        e = src.word(5 + hj);
        const uint32_t nl = e & 0xffffu, lb = nl < 63 ? nl : 63;
        if ((lb < 32 ? h.name_len_lo >> lb : h.name_len_hi >> (lb - 32)) & 1u) break;
        hp += nl + (e >> 16);  // no rule references a header name of this length
      }
      if (!__any(hj < nhdr)) break;
      if (hj < nhdr) {
        const uint32_t nl = e & 0xffffu, vl = e >> 16;
        if (h.lds_name_tab != kNone) {
          f = name_field_of(c, h, src, hp, nl);
        } else {
          const uint32_t code = walk_dfa<false, false>(c, h.n_dfas, src, hp, nl);
          if (code & kLatchedBit) f = 3u + (code & ~kLatchedBit);
          else if (code) f = c.name_field[code];
        }
        if (f != kNone && ((present >> f) & 1ull)) f = kNone;  // first occurrence wins
        p = hp + nl;
        len = vl;
        hp += nl + vl;
        ++hj;
      }
    }
    HPROF(2);  // job selection, header-name lookup
    if (f != kNone) {
      present |= 1ull << f;
      const FieldDesc& fd = c.fields[f];
      uint32_t kend = fd.ndfa;
      if constexpr (kReg < 0) {
        if (fd.gram_tab != kNone) {
          // the search groups the value's grams select, up to four chains at a
          // time (per lane: its own groups); the packed groups before them below
          const uint32_t sel = gram_select(c, fd, src, p, len), ns = fd.n_search;
          HPROF(6);  // (diagnostic build) the gram filter
          uint64_t selm = ns > 32 ? (static_cast<uint64_t>(sel) << 32 | sel) : sel;
          if (ns < 64) selm &= (1ull << ns) - 1;
          while (__any(selm != 0)) {
            uint32_t dl[kSearchChains], m = 0;
#pragma unroll
            for (uint32_t j = 0; j < kSearchChains; ++j) {
              dl[j] = fd.dfa_first + fd.search_first + (selm ? static_cast<uint32_t>(__builtin_ctzll(selm)) : 0u);
              m = selm ? j + 1 : m;
              selm &= selm - 1;
            }
            uint32_t out[kSearchChains];
            walk_search4v<false>(c, dl, m, src, p, len, out);  // (LDS-resident tables keep a program copy)
#pragma unroll
            for (uint32_t j = 0; j < kSearchChains; ++j)
              if (j < m) codes.set(dl[j], out[j]);
          }
          HPROF(3);  // gram filter + the selected groups' walks
          kend = fd.search_first;
        }
        if (fd.alit_tab != kNone) alit_scan(c, fd, src, p, len, codes);
      }
      for (uint32_t k = 0; k < kend; ++k) {
        const uint32_t d = fd.dfa_first + k;
        if constexpr (kReg < 0) {
          if (c.dds[d].kind == kDfaAlit) continue;  // (alit_scan)
          if (c.dds[d].kind == kDfaSearch && k + 1 < kend && c.dds[d + 1].kind == kDfaSearch) {
            // a run of search automata, four at a time (a single one below:
            // walk_search, which reads an LDS-resident table from LDS)
            uint32_t m = 1;
            while (m < kSearchChains && k + m < kend && c.dds[d + m].kind == kDfaSearch) ++m;
            uint32_t out[kSearchChains];
            walk_search4<false>(c, d, m, src, p, len, out);
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
              if (j < m) codes.set(d + j, out[j]);
            k += m - 1;
            continue;
          }
        }
        const uint32_t code = walk_dfa<kLit, (kReg < 0)>(c, d, src, p, len);
        HPROF(3);  // the walk, end code included
        codes.set(d, code);
        touch(d, code);
      }
      if constexpr (kDcap)
        for (uint32_t m = fd.dcap_mask; m; m &= m - 1) {
          const uint32_t k = static_cast<uint32_t>(__builtin_ctz(m));
          if (dcap_holds<kLit>(c, dspec[k], src, p, len)) dcap |= 1u << k;
        }
    }
  }

  HPROF(5);
  if constexpr (kAblate == 1) {
    uint32_t acc = static_cast<uint32_t>(present);
    for (uint32_t d = 0; d < h.n_dfas; ++d) acc += codes.get(d);
    return static_cast<int32_t>(acc & 7u);
  }
  o.present = present;
  o.ex = ex;
  o.e0 = e0;
  o.h0 = h0;
  o.remote = w1;
  o.pf_t = pf_t;
  o.dcap = dcap;
  return kNeedVerify;
}

// Verification phase: the first rule (smallest index) among the keyed
// candidates whose other matchers, port entry and remote set hold; the
// check-record lists are selected by the walks' end codes.
// kSlowPass (http_slow_kernel): rules with slow-path matchers (kCrSlow) are
// decided by the executor of regex_vm.h on the record's field values (src,
// vm: this lane's scratch); in the first pass such a rule whose automaton
// checks pass only marks the request for deferral.
template <int kReg, int kSlowPass = 0, bool kDcap = false, class Src = GlbSrc>
__device__ __forceinline__ int32_t eval_verify(const Ctx& c, const HttpHeader& h, const WalkOut<kReg>& o,
                                               const Src* src = nullptr, uint32_t* vm = nullptr) {
  const Codes<kReg>& codes = o.codes;
  const uint64_t present = o.present;
  asm volatile("" ::"v"(o.pf_t));  // the touch completes here, not at its first use
  const uint32_t ex = o.ex, e0 = o.e0, remote = o.remote;
  const bool h0 = o.h0;
  const uint32_t dcap = o.dcap;
  // a matcher on a forced-capture pattern (pattern word >> kDcapShift = k + 1)
  // also needs that pattern's byte checks to have held (program.h DcapSpec)
  auto dcap_ok = [&](uint32_t pat) -> bool {
    if constexpr (!kDcap) return true;
    const uint32_t k = pat >> kDcapShift;
    return k == 0 || ((dcap >> (k - 1)) & 1u) != 0;
  };
  // (pattern words carry dcap ids only in programs with forced captures)
  auto pm = [](uint32_t pat) -> uint32_t { return kDcap ? (pat & kPatMask) : pat; };
  // a rule may decide only if it belongs to ex, or to e0 when e0 has HTTP rules
  auto eligible = [&](uint32_t hd) -> bool {
    const uint32_t e = cr_entry(hd);
    return e == ex || (h0 && e == e0);
  };
  const bool masked = h.n_dfas <= 64;
  const uint64_t cand_all = masked ? ((static_cast<uint64_t>(h.cand_dfas_hi) << 32) | h.cand_dfas_lo) : 0;
  uint32_t best = h.always_rule;
  uint32_t min_slow = kNone;   // first pass: smallest slow-path rule whose automaton checks passed
  uint32_t min_limit = kNone;  // slow pass: smallest rule whose evaluation hit the executor's limits
  // A candidate whose checks passed: rules with slow-path matchers are
  // deferred (first pass) or run through the executor (slow pass).
  auto take = [&](uint32_t rid, uint32_t hd) -> bool {
    if (!(hd & kCrSlow)) {
      best = rid;
      return true;
    }
    if constexpr (!kSlowPass) {
      min_slow = rid < min_slow ? rid : min_slow;
      return false;
    } else {
      const uint32_t* sl = c.prog + h.off_slow + 2u * rid;
      const uint32_t so = sl[0], sn = sl[1];
      bool all = true;
      for (uint32_t q = 0; q < sn && all; ++q) {
        const uint32_t f = c.pool[so + 2 * q], off = c.pool[so + 2 * q + 1];
        uint32_t pos = 0, len = 0;
        if (!field_at(c, h, *src, f, &pos, &len)) {
          all = false;
          break;
        }
        const int r = vm_match(c.prog + off, reinterpret_cast<const uint8_t*>(src->w) + pos, len, vm,
                               kSlowPass == 1 ? kVmScratchWords : kVmScratchWords2,
                               kSlowPass == 1 ? kVmMaxSteps : kVmMaxSteps2);
        if (r < 0) min_limit = rid < min_limit ? rid : min_limit;  // kVmLimit / kVmDeep
        all = r == kVmMatched;
      }
      if (all) best = rid;
      return all;
    }
  };
  auto remote_ok = [&](uint32_t rid) -> bool {  // PortNetworkPolicyRule::Matches (h:92-97)
    const uint32_t* rp = reinterpret_cast<const uint32_t*>(c.remotes + rid);
    uint32_t roff = gld(rp), rlen = gld(rp + 1);
    asm volatile("" : "+v"(roff), "+v"(rlen));
    uint32_t lo = 0, hi = rlen;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (gld_now(c.pool + roff + mid) < remote) lo = mid + 1;
      else hi = mid;
    }
    return lo < rlen && gld_now(c.pool + roff + lo) == remote;
  };
  auto scan = [&](Span cl) {
    uint32_t o = cl.off;
    for (uint32_t j = 0; j < cl.len; ++j) {
      // one record: rid, header, up to 3 matchers fetched together
      uint32_t rw[8];
#pragma unroll
      for (uint32_t q = 0; q < 8; ++q) rw[q] = gld(c.cr + o + q);
      asm volatile("" : "+v"(rw[0]), "+v"(rw[1]), "+v"(rw[2]), "+v"(rw[3]), "+v"(rw[4]), "+v"(rw[5]), "+v"(rw[6]),
                   "+v"(rw[7]));
      const uint32_t rid = rw[0], nm = cr_matchers(rw[1]);
      if (rid >= best) break;
      bool ok = eligible(rw[1]) && (!(rw[1] & kCrRemote) || remote_ok(rid));
      for (uint32_t q = 0; q < nm && ok; ++q) {
        const uint32_t a = q < 3 ? (q == 0 ? rw[2] : q == 1 ? rw[4] : rw[6]) : gld_now(c.cr + o + 2 + 2 * q);
        const uint32_t pat = q < 3 ? (q == 0 ? rw[3] : q == 1 ? rw[5] : rw[7]) : gld_now(c.cr + o + 3 + 2 * q);
        const uint32_t f = a & 0xffu;
        if (!((present >> f) & 1ull)) ok = false;
        else if (!((a >> 8) & 1u))
          ok = code_has<(kReg < 0)>(c, a >> 9, codes.get(a >> 9), pm(pat)) && dcap_ok(pat);
      }
      if (ok && take(rid, rw[1])) break;
      o += 2 + 2 * nm;
    }
  };
  // Candidates of each DFA end code: one 64-byte CandEntry whose first check
  // record is inline; longer lists fall back to the pool scan.
  auto check_entry = [&](const u32x4 q0, const u32x4 q1, const u32x4 q2) {  // a CandEntry's first 48 bytes
    const uint32_t len = q0.x, rid = q0.z, hd = q0.w, nm = cr_matchers(hd);  // len, off, rid, hdr
    if (len == 1 && nm <= kCandInlineMatchers) {
      if (rid >= best) return;
      const uint32_t ma[4] = {q1.x, q1.z, q2.x, q2.z}, mp[4] = {q1.y, q1.w, q2.y, q2.w};
      bool ok = eligible(hd) && (!(hd & kCrRemote) || remote_ok(rid));
      if constexpr (kReg < 0) {  // search programs (mask codes): one matcher after the other
#pragma unroll
        for (uint32_t q = 0; q < kCandInlineMatchers; ++q) {
          if (q < nm && ok) {
            const uint32_t a = ma[q];
            if (!((present >> (a & 0xffu)) & 1ull)) ok = false;
            else if (!((a >> 8) & 1u))
              ok = code_has<(kReg < 0)>(c, a >> 9, codes.get(a >> 9), pm(mp[q])) && dcap_ok(mp[q]);
          }
        }
      } else {
        // The inline matchers in two rounds of independent LDS reads (each
        // DFA's mask table, then the set's mask word) instead of one dependent
        // chain per matcher; set codes whose masks are not in LDS take the
        // general code_has.
        uint32_t cq[4], mo[4], w[4];
        bool need[4], set[4];
#pragma unroll
        for (uint32_t q = 0; q < kCandInlineMatchers; ++q) {  // round 1: the DFAs' mask tables
          const uint32_t a = ma[q];
          cq[q] = q < nm ? codes.get(a >> 9) : 0u;
          need[q] = q < nm && !((a >> 8) & 1u);  // a code matcher (else presence only)
          set[q] = need[q] && cq[q] && !(cq[q] & kLatchedBit);
          mo[q] = lld(reinterpret_cast<const uint32_t*>(c.dds + (a >> 9)) + offsetof(DfaDesc, lds_mask) / 4);
        }
#pragma unroll
        for (uint32_t q = 0; q < kCandInlineMatchers; ++q) {  // round 2: the sets' mask words
          const bool rd = set[q] && mo[q] != kNone;
          w[q] = lld(c.img + (rd ? mo[q] + 2u * cq[q] + (pm(mp[q]) >> 5) : 0u));
        }
        bool slow = false;
#pragma unroll
        for (uint32_t q = 0; q < kCandInlineMatchers; ++q) {
          const uint32_t a = ma[q], p = pm(mp[q]);
          const bool pres = q >= nm || ((present >> (a & 0xffu)) & 1ull);
          const bool lat = (cq[q] & kLatchedBit) != 0;
          const bool hit = !need[q] || (cq[q] != 0 && dcap_ok(mp[q]) &&
                                        (lat ? (cq[q] & ~kLatchedBit) == p
                                             : (mo[q] == kNone || ((w[q] >> (p & 31u)) & 1u))));
          slow |= set[q] && mo[q] == kNone;
          ok = ok && pres && hit;
        }
        if (slow && ok) {  // rare: sets whose masks are in the program pool
#pragma unroll
          for (uint32_t q = 0; q < kCandInlineMatchers; ++q) {
            if (q < nm && ok && need[q] && cq[q] && !(cq[q] & kLatchedBit) && mo[q] == kNone)
              ok = code_has<(kReg < 0)>(c, ma[q] >> 9, cq[q], pm(mp[q]));
          }
        }
      }
      if (ok) take(rid, hd);
    } else {
      scan(Span{q0.y, len});
    }
  };
  auto check_inline = [&](const uint32_t* e) {  // e -> CandEntry in LDS
    const u32x4* q = reinterpret_cast<const u32x4*>(e);
    check_entry(q[0], q[1], q[2]);
  };
  // only DFAs with candidate entries (search programs: only those the record
  // set a code for -- a handful of dozens)
  uint64_t cm = cand_all;
  if constexpr (kReg < 0) cm &= codes.masked ? codes.valid : ~0ull;
  for (uint32_t i = 0; masked ? cm != 0 : i < h.n_dfas; ++i) {
    uint32_t d = i;
    if (masked) {
      d = static_cast<uint32_t>(__builtin_ctzll(cm));
      cm &= cm - 1;
    }
    const uint32_t code = codes.get(d);
    if (!code) continue;
    const DfaDesc& dd = c.dds[d];
    if (kReg < 0 && dd.kind != kDfaPacked) {  // search / alit: candidates of every matched pattern (entry p)
      for (uint32_t m = code; m; m &= m - 1) {
        const uint32_t idx = static_cast<uint32_t>(__builtin_ctz(m));
        const uint32_t mw = dd.lds_ctmask != kNone ? lld(c.img + dd.lds_ctmask + (idx >> 5))
                                                   : gld_now(c.prog + dd.ctmask_off + (idx >> 5));
        if (!((mw >> (idx & 31u)) & 1u)) continue;
        if (dd.lds_ct != kNone) {
          check_inline(c.img + dd.lds_ct + 16u * idx);
        } else {
          typedef __attribute__((address_space(1))) const u32x4* gq;
          const gq q = (gq)(c.prog + dd.ct_off + 16u * idx);
          u32x4 q0 = q[0], q1 = q[1], q2 = q[2];
          asm volatile("" : "+v"(q0), "+v"(q1), "+v"(q2));
          check_entry(q0, q1, q2);
        }
      }
      continue;
    }
    const uint32_t idx = (code & kLatchedBit) ? dd.nsets + (code & ~kLatchedBit) : code;
    const uint32_t mw =
        dd.lds_ctmask != kNone ? lld(c.img + dd.lds_ctmask + (idx >> 5)) : gld(c.prog + dd.ctmask_off + (idx >> 5));
    if (!((mw >> (idx & 31u)) & 1u)) continue;  // no candidates
    if (dd.lds_ct != kNone) {
      check_inline(c.img + dd.lds_ct + 16u * idx);
    } else {  // an HBM candidate entry (touched by the walk phase)
      typedef __attribute__((address_space(1))) const u32x4* gq;
      const gq q = (gq)(c.prog + dd.ct_off + 16u * idx);
      u32x4 q0 = q[0], q1 = q[1], q2 = q[2];
      asm volatile("" : "+v"(q0), "+v"(q1), "+v"(q2));
      check_entry(q0, q1, q2);
    }
  }
  for (uint64_t pm = ((static_cast<uint64_t>(h.pres_fields_hi) << 32) | h.pres_fields_lo) & present; pm;
       pm &= pm - 1) {
    const uint32_t f = static_cast<uint32_t>(__builtin_ctzll(pm));
    scan(c.fields[f].presence);
  }
  if (h.zero_list.len) scan(h.zero_list);

  if (!kSlowPass && min_slow < best) return kDeferred;
  // undecided before the first match: the second tier runs it with the large
  // stack and step budget; past those the verdict is "unsupported"
  if (kSlowPass && min_limit < best) return kSlowPass == 1 ? kDeferred2 : L7M_VERDICT_UNSUPPORTED;
  if (best != kNone) return static_cast<int32_t>(best);
  // the exact-port entry matched nothing; a port-0 entry without HTTP rules allows
  return h0 ? L7M_VERDICT_DENY : L7M_VERDICT_ALLOW_NO_L7;
}

// A wave-uniform lane's 64-bit value: v_readlane (no LDS round trip, unlike
// the ds_bpermute of __shfl); `src` must be wave-uniform.
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t src) {
  const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), src);
  const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), src);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
  const uint32_t lo = __shfl(static_cast<uint32_t>(v), src);
  const uint32_t hi = __shfl(static_cast<uint32_t>(v >> 32), src);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Per-rule hit counters: none, per-workgroup LDS counters flushed once at the
// end (small rule sets), or wave-aggregated global atomics.
enum HitMode { kNoHits = 0, kLdsHits = 1, kGlobalHits = 2 };

// kLit: the program has literal tables (DfaDesc::lit_tab) for HBM-walked
// DFAs; a separate instantiation, so programs without them keep the leaner
// walk code.
#if L7M_HTTP_WG_PER_CU > 1
// (experiment) several workgroups per CU: the register budget of their waves
#define L7M_HTTP_OCC __attribute__((amdgpu_waves_per_eu(L7M_HTTP_WG_PER_CU * L7M_HTTP_WAVES / 4)))
#else
#define L7M_HTTP_OCC
#endif
// The evaluation of one batch by one workgroup, `part` of `nparts` of the
// grid; each wave takes share wave_index of wave_count (load_image false
// would keep an LDS image already in place).
template <int kHits, int kReg, int kAblate, int kFeat>
__device__ __forceinline__ void http_eval_body(const uint32_t* __restrict__ prog, const uint8_t* __restrict__ arena,
                                               uint64_t arena_bytes, const uint64_t* __restrict__ offs, uint64_t n,
                                               int32_t* __restrict__ verdicts, unsigned long long* __restrict__ hits,
                                               uint32_t stage, uint32_t* __restrict__ scratch,
                                               uint32_t* __restrict__ slowq, bool load_image, uint32_t part,
                                               uint32_t nparts, uint32_t wave_index, uint32_t wave_count,
                                               DoneSignal done = DoneSignal{nullptr, nullptr, 0},
                                               uint32_t* __restrict__ hslice = nullptr) {
  extern __shared__ __align__(16) uint32_t smem[];
  const HttpHeader& h = *reinterpret_cast<const HttpHeader*>(prog);
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  uint32_t* img = smem;
  const uint32_t n_ctr = h.n_rules + 2;
  // hit counters (kLdsHits): LDS, or (kSliceHits) this workgroup's global slice
  uint32_t* ctr = kSliceHits ? hslice + static_cast<uint64_t>(part) * ((n_ctr + 63u) & ~63u) : smem + h.lds_image_words;
  uint32_t* col = (kSliceHits ? smem + h.lds_image_words : ctr) +
                  (kHits == kLdsHits && !kSliceHits ? ((n_ctr + 3u) & ~3u) : 0u);  // LDS code columns (!kReg)
  uint8_t* stg = reinterpret_cast<uint8_t*>(col + (kReg ? 0u : h.n_dfas * kBlock)) + wv * (stage + 16u);
  // This wave's contiguous share of the batch, consumed in tiles of <= 64
  // records (wave wave_index of wave_count).  The first tile's offsets are
  // requested before the LDS image is loaded, so the two latencies overlap
  // (small batches: the offsets may sit in pinned host memory, across PCIe).
  const uint64_t gw = wave_index;
  const uint64_t nw = wave_count;
#if L7M_SPEC_TILE
  // (kSpecTile) a small batcher batch: wave 0 takes it whole
  const bool spec = done.flag && n <= 64 && arena_bytes <= stage;
  const uint64_t start = spec ? 0 : n * gw / nw;
  const uint64_t end = spec ? (gw == 0 ? n : 0) : n * (gw + 1) / nw;
#else
  const uint64_t end = n * (gw + 1) / nw;
#define start (n * gw / nw)
#endif
  auto load_offs = [&](uint64_t cur, uint64_t* o, uint64_t* onext) {
    *o = 0;
    *onext = 0;
    if (cur < end && lane < end - cur) {
      *o = offs[cur + lane];
      *onext = cur + lane + 1 < n ? offs[cur + lane + 1] : arena_bytes;
    }
  };
  uint64_t o1, n1, o2, n2;
  load_offs(start, &o1, &n1);
#if L7M_SPEC_TILE
  if (spec && gw == 0) {
    // the batch's bytes from offset 0, before the offsets (pinned host
    // memory: both requests cross PCIe; plan() below checks the guess)
    const u32x4* src = reinterpret_cast<const u32x4*>(arena);
#pragma unroll
    for (uint32_t it = 0; it < kCopyIters; ++it) {
      const uint32_t q = it * 64u + lane;
      if (q * 16u < arena_bytes)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + q),
                                         reinterpret_cast<__attribute__((address_space(3))) void*>(
                                             reinterpret_cast<uintptr_t>(stg + it * 1024u)),
                                         16, 0, 2);
    }
  }
#endif
  if (load_image) {
    const uint4* g = reinterpret_cast<const uint4*>(prog + h.lds_image_off);
    uint4* l = reinterpret_cast<uint4*>(img);
    for (uint32_t i = tid; i < h.lds_image_words / 4u; i += kBlock) l[i] = g[i];
  }
  if (kHits == kLdsHits)
    for (uint32_t i = tid; i < n_ctr; i += kBlock) {
      if constexpr (kSliceHits) __hip_atomic_store(ctr + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else ctr[i] = 0;
    }
  __syncthreads();

  Ctx c;
  c.prog = prog;
  c.img = img;
  c.dds = reinterpret_cast<const DfaDesc*>(img + h.lds_dfas);
  c.fields = reinterpret_cast<const FieldDesc*>(img + h.lds_fields);
  c.name_field = img + h.lds_name_field;
  c.sets = reinterpret_cast<const Span*>(prog + h.off_sets);
  c.pool = prog + h.off_pool;
  c.cr = prog + h.off_cr;
  c.remotes = reinterpret_cast<const Span*>(prog + h.off_remotes);
  uint32_t* mycol = col + tid;
  // diagnostic wave timeline per tile (kProf, s_memtime): [0] top wait,
  // [1] walks, [2] entry wait, [3] issue, [4] verify + store, [5] counters;
  // [6] tiles
  uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t prof_tile = 0, te0 = 0;
  uint64_t qt[7] = {0, 0, 0, 0, 0, 0, 0}, qlast = kProf ? __builtin_amdgcn_s_memtime() : 0;
  auto qtn = [&](int i) {
    if constexpr (kProf) {
      const uint64_t t_ = __builtin_amdgcn_s_memtime();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      qt[i] += t_ - qlast;
      qlast = t_;
    }
  };

  // Software pipeline per wave: while tile t is evaluated from the LDS
  // stage, tile t+1's bytes and tile t+2's offsets are already in flight.
  struct Tile {
    uint64_t cur, o, onext, base;
    uint32_t k, bytes, take;
  };
  auto plan = [&](uint64_t cur, uint64_t o, uint64_t onext) -> Tile {
    Tile t;
    t.cur = cur;
    t.o = o;
    t.onext = onext;
    if (cur >= end) {
      t.base = 0;
      t.k = t.bytes = t.take = 0;
      return t;
    }
    const uint64_t m = end - cur < 64 ? end - cur : 64;
    const uint64_t o0 = readlane64(o, 0);
    t.base = o0 & ~15ull;
    // Leading run of records that lie, in order, inside a window <= stage.
    const bool ok = lane < m && (o & 3) == 0 && o >= o0 && onext >= o && onext <= arena_bytes &&
                    onext - t.base <= stage;
    const uint64_t okm = __ballot(ok);
    t.k = okm == ~0ull ? 64u : static_cast<uint32_t>(__builtin_ctzll(~okm));
    t.bytes = t.k ? static_cast<uint32_t>(readlane64(onext, t.k - 1) - t.base) : 0u;
    // A stage that holds fewer than half a tile of records (large records,
    // config 5: 7-12 of 64) would leave most lanes idle: the tile then takes
    // all m records and lanes past the staged run read theirs from HBM.
    t.take = t.k >= kMinStagedTake ? t.k : static_cast<uint32_t>(m);
    return t;
  };
  // Staging by LDS-DMA (global_load_lds_dwordx4, non-temporal): the next
  // tile's bytes go HBM -> the wave's stage with no VGPR destination and no
  // ds_write pass (lane l of piece `it` lands at stage + it * 1 KiB + 16 l,
  // the coalesced copy's own layout), issued after the walks, the stage's
  // only readers.  (Register staging measured 3.52 vs 3.47-3.49 ms on config
  // 2, 8.93 vs 8.83 on config 4: profiles/r03/ab_round3.md.)
  auto issue_bytes = [&](const Tile& t) {
    const u32x4* src = reinterpret_cast<const u32x4*>(arena + t.base);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this tile's stage reads are done
#pragma unroll
    for (uint32_t it = 0; it < kCopyIters; ++it) {
      const uint32_t q = it * 64u + lane;
      if (q * 16u < t.bytes)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + q),
                                         reinterpret_cast<__attribute__((address_space(3))) void*>(
                                             reinterpret_cast<uintptr_t>(stg + it * 1024u)),
                                         16, 0, 2);
    }
    // L2 prefetch of the first lines of the records this tile's lanes will
    // read from HBM (the lanes past the staged run): 4-byte LDS-DMA loads
    // into a scratch corner at the end of the stage (config 5: 0.555 ->
    // 0.545 ms, profiles/r04/ab_round4.md; no effect where tiles are staged)
    if (t.take > t.k && t.bytes + 256u <= stage) {
      const bool hbm = lane >= t.k && lane < t.take;
      const uint64_t o = t.o & ~3ull, len = t.onext > t.o ? t.onext - t.o : 0;
      auto* junk = reinterpret_cast<__attribute__((address_space(3))) void*>(
          reinterpret_cast<uintptr_t>(stg + stage - 256u));
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j)
        if (hbm && 128ull * j < len && o + 128ull * j + 4 <= arena_bytes)
          __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(arena + o + 128ull * j), junk, 4, 0, 0);
    }
  };
  Tile t = plan(start, o1, n1);
#if L7M_SPEC_TILE
  if (!(spec && t.base == 0 && t.take == t.k)) {  // (a tile at offset 0 is what the guess requested)
    if (spec) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the guessed bytes have landed first
    issue_bytes(t);
  }
#else
#undef start
  issue_bytes(t);
#endif
  load_offs(t.cur + t.take, &o2, &n2);
  while (t.cur < end) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tile's LDS-DMA pieces have landed
    wave_sync();
    qtn(0);

    const uint64_t o = t.o, onext = t.onext, base = t.base;
    const uint32_t k = t.k, take = t.take;
    int32_t v = 0;
    if constexpr (kProf) te0 = __builtin_amdgcn_s_memtime();
    WalkOut<kReg> wo;
    if constexpr (!kReg) wo.codes.p = mycol;
    if constexpr (kReg < 0) {  // search programs: the codes live in the global scratch
      wo.codes.p = scratch + static_cast<uint64_t>(part) * kBlock + tid;
      wo.codes.stride = nparts * kBlock;
    }
    if (lane < take) {
      bool done = false;
      if (lane < k && onext - o >= L7M_HTTP_REC_FIXED) {
        const LdsSrc s{reinterpret_cast<const uint32_t*>(stg + (o - base))};
        const uint32_t w0 = s.word(0);
        if (((static_cast<uint64_t>(w0) + 3) & ~3ull) <= onext - o) {
          v = eval_walk<kReg, kAblate, kFeat>(c, h, s, onext - o, wo, prof);
          done = true;
        }
      }
      if (!done) {  // outside the staged window: read HBM directly
        const bool inb = (o & 3) == 0 && o + L7M_HTTP_REC_FIXED <= arena_bytes;
        const GlbSrc s{reinterpret_cast<const uint32_t*>(arena + (inb ? o : 0))};
        v = inb ? eval_walk<kReg, kAblate, kFeat>(c, h, s, arena_bytes - o, wo, prof) : L7M_VERDICT_PARSE_ERROR;
      }
    }
    qtn(1);
    qtn(2);
    // The next tile's bytes are requested only now, after the walks: they
    // land during verification without holding kCopyIters x 4 registers
    // through the walks (the walks read LDS only).
    const Tile t2 = plan(t.cur + t.take, o2, n2);
    issue_bytes(t2);
    load_offs(t2.cur + t2.take, &o2, &n2);
    qtn(3);
    if (lane < take) {
      if (v == kNeedVerify) v = eval_verify<kReg, 0, (kFeat & kFeatDcap) != 0>(c, h, wo);
      verdicts[t.cur + lane] = v;
      if (v == kDeferred) {  // decided by http_slow_kernel (rules with slow-path matchers)
        const uint32_t at = atomicAdd(slowq, 1u);
        slowq[1 + at] = static_cast<uint32_t>(t.cur + lane);
      }
    }
    qtn(4);
    if constexpr (kProf) prof_tile += __builtin_amdgcn_s_memtime() - te0;
    if (kHits != kNoHits) {
      uint32_t slot = kNone;
      // allows decided without a rule (no L7 rules, no port policy) are not counted
      if (lane < take && v < L7M_VERDICT_ALLOW_NO_PORT_POLICY && v != kDeferred)
        slot = v >= 0 ? static_cast<uint32_t>(v) + 2u : (v == L7M_VERDICT_DENY ? 0u : 1u);
      if (kHits == kLdsHits) {
        // denies / errors are common: one add per wave for them
        const uint64_t dm = __ballot(slot == 0u), em = __ballot(slot == 1u);
        auto add = [&](uint32_t i, uint32_t x) {
          if constexpr (kSliceHits) (void)__hip_atomic_fetch_add(ctr + i, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          else atomicAdd(ctr + i, x);
        };
        if (lane == 0 && dm) add(0, static_cast<uint32_t>(__popcll(dm)));
        if (lane == 0 && em) add(1, static_cast<uint32_t>(__popcll(em)));
        if (slot != kNone && slot >= 2u) add(slot, 1u);
      } else {
        count_slot(hits, slot, slot != kNone);
      }
    }
    wave_sync();  // the stage is overwritten by the next tile
    t = t2;
    qtn(5);
    qt[6] += 1;
  }
  if (kProf && ((part == 0 && wv == 0) || (part == 101 && wv == 7))) {
    if (lane == 0)
      printf("L7M_QT block %u wave %u tiles %llu cycles/tile: topwait %llu walks %llu entry %llu issue %llu "
             "verify %llu counters %llu\n",
             part, wv, (unsigned long long)qt[6], (unsigned long long)(qt[0] / (qt[6] ? qt[6] : 1)),
             (unsigned long long)(qt[1] / (qt[6] ? qt[6] : 1)), (unsigned long long)(qt[2] / (qt[6] ? qt[6] : 1)),
             (unsigned long long)(qt[3] / (qt[6] ? qt[6] : 1)), (unsigned long long)(qt[4] / (qt[6] ? qt[6] : 1)),
             (unsigned long long)(qt[5] / (qt[6] ? qt[6] : 1)));
    prof[7] = prof_tile;
    for (int q = 1; q < 8; ++q)
      for (uint32_t m = 1; m < 64; m <<= 1) {
        const uint64_t o2 = shfl64(prof[q], lane ^ m);
        prof[q] = o2 > prof[q] ? o2 : prof[q];
      }
    if (lane == 0)
      printf("L7M_PROF validate %llu jobsel %llu walks %llu setcode %llu tail %llu gram %llu eval %llu\n",
             (unsigned long long)prof[1], (unsigned long long)prof[2], (unsigned long long)prof[3],
             (unsigned long long)prof[4], (unsigned long long)prof[5], (unsigned long long)prof[6],
             (unsigned long long)prof[7]);
  }
  if (kHits == kLdsHits) {
    __syncthreads();
    for (uint32_t i = tid; i < n_ctr; i += kBlock) {
      const uint32_t x = kSliceHits ? __hip_atomic_load(ctr + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ctr[i];
      if (x) atomicAdd(hits + i, static_cast<unsigned long long>(x));
    }
  }
#if L7M_SPEC_TILE
  if (spec && kHits == kNoHits) {
    // wave 0 decided the whole batch: it alone signals (no counter round trip)
    if (gw == 0) {
      __threadfence_system();
      if (lane == 0) __hip_atomic_store(done.flag, done.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
#endif
  if (done.flag) {  // (l7m_device.h DoneSignal)
    __threadfence_system();  // this wave's verdict stores (and counters) are visible system-wide
    if (lane == 0 && atomicAdd(done.ctr, 1u) == wave_count - 1u) {
      __threadfence_system();
      __hip_atomic_store(done.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done.flag, done.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <int kHits, int kReg, int kAblate, int kFeat>
__global__ __launch_bounds__(kBlock) L7M_HTTP_OCC void http_eval_kernel(const uint32_t* __restrict__ prog,
                                                           const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                           const uint64_t* __restrict__ offs, uint64_t n,
                                                           int32_t* __restrict__ verdicts,
                                                           unsigned long long* __restrict__ hits, uint32_t stage,
                                                           uint32_t* __restrict__ scratch, uint32_t* __restrict__ slowq,
                                                           DoneSignal done, uint32_t* __restrict__ hslice) {
  http_eval_body<kHits, kReg, kAblate, kFeat>(prog, arena, arena_bytes, offs, n, verdicts, hits, stage, scratch, slowq,
                                             true, blockIdx.x, gridDim.x, blockIdx.x * kWaves + (threadIdx.x >> 6),
                                             gridDim.x * kWaves, done, hslice);
}

// Second pass over the requests the first pass deferred (a slow-path rule may
// decide them, program.h kCrSlow): one lane per queued request, the same walk
// phase, then verification with the slow-path executor (regex_vm.h) on this
// lane's scratch.  Each wave takes the next 64 queued requests from a work
// counter and copies every record that fits kSlowRec bytes into its lane's
// LDS slot (walk and executor then read LDS; larger records are read from
// HBM).  Two tiers (regex_vm.h): tier 1 runs every deferred request with 16
// KiB of executor stack, kSlowWavesPerCu waves per CU; requests it could not
// decide (stack or step budget) are queued for tier 2, kSlowBlocks2 waves
// with 1 MiB per lane.  Verdicts and counters of these requests are written
// here only.
constexpr uint32_t kSlowBlock = 64;       // one wave per workgroup
constexpr uint32_t kSlowWavesPerCu = 4;   // tier 1
constexpr uint32_t kSlowBlocks2 = 4;      // tier 2: 256 lanes x 1 MiB
constexpr uint32_t kSlowRec = 256;        // LDS record slot per lane (records <= kSlowRec - 32 bytes)

// LDS of one slow-pass workgroup: the table image, the end-code columns
// (Codes<0>, first-pass stride), the record slots.
inline size_t http_slow_lds_bytes(const HttpHeader& h, bool reg) {
  return 4u * (static_cast<size_t>(h.lds_image_words) + (reg ? 0u : static_cast<size_t>(h.n_dfas) * kBlock)) +
         static_cast<size_t>(kSlowBlock) * kSlowRec;
}

template <int kReg, int kFeat, int kTier>
__global__ __launch_bounds__(kSlowBlock) void http_slow_kernel(const uint32_t* __restrict__ prog,
                                                               const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                               const uint64_t* __restrict__ offs, uint64_t n,
                                                               int32_t* __restrict__ verdicts,
                                                               unsigned long long* __restrict__ hits,
                                                               const uint32_t* __restrict__ slowq,
                                                               uint32_t* __restrict__ slowq2,
                                                               uint32_t* __restrict__ vmscratch,
                                                               uint32_t* __restrict__ work) {
  extern __shared__ __align__(16) uint32_t smem[];
  const HttpHeader& h = *reinterpret_cast<const HttpHeader*>(prog);
  const uint32_t tid = threadIdx.x;
  uint32_t* img = smem;
  {
    const uint4* g = reinterpret_cast<const uint4*>(prog + h.lds_image_off);
    uint4* l = reinterpret_cast<uint4*>(img);
    for (uint32_t i = tid; i < h.lds_image_words / 4u; i += kSlowBlock) l[i] = g[i];
  }
  __syncthreads();
  Ctx c;
  c.prog = prog;
  c.img = img;
  c.dds = reinterpret_cast<const DfaDesc*>(img + h.lds_dfas);
  c.fields = reinterpret_cast<const FieldDesc*>(img + h.lds_fields);
  c.name_field = img + h.lds_name_field;
  c.sets = reinterpret_cast<const Span*>(prog + h.off_sets);
  c.pool = prog + h.off_pool;
  c.cr = prog + h.off_cr;
  c.remotes = reinterpret_cast<const Span*>(prog + h.off_remotes);
  uint32_t* slot = img + h.lds_image_words + (kReg ? 0u : h.n_dfas * kBlock) + tid * (kSlowRec / 4);
  const uint32_t gtid = blockIdx.x * kSlowBlock + tid;
  uint32_t* vm = vmscratch + static_cast<uint64_t>(gtid) * (kTier == 1 ? kVmScratchWords : kVmScratchWords2);
  const uint32_t* q_in = kTier == 1 ? slowq : slowq2;
  const uint32_t nq = q_in[0];
  uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (;;) {
    uint32_t base = 0;
    if (tid == 0) base = atomicAdd(work, kSlowBlock);
    base = __shfl(base, 0);
    if (base >= nq) break;
    const uint32_t q = base + tid;
    const uint32_t ri = q < nq ? q_in[1 + q] : kNone;
    int32_t v = kDeferred;  // (inactive lanes)
    if (ri < n) {
      const uint64_t o = offs[ri];
      WalkOut<kReg> wo;
      if constexpr (!kReg) wo.codes.p = img + h.lds_image_words + tid;
      v = L7M_VERDICT_PARSE_ERROR;
      const bool inb = (o & 3) == 0 && o + L7M_HTTP_REC_FIXED <= arena_bytes;
      const uint32_t* rw = reinterpret_cast<const uint32_t*>(arena + (inb ? o : 0));
      const uint32_t rlen = inb ? ((rw[0] + 3u) & ~3u) : 0u;
      if (inb && rlen <= kSlowRec - 32 && o + rlen <= arena_bytes) {
        // the record into this lane's LDS slot (16-byte loads; the slack past
        // it is zero so over-reads see no stale bytes)
        const uint4* g = reinterpret_cast<const uint4*>(rw);
        uint4* l = reinterpret_cast<uint4*>(slot);
        for (uint32_t i = 0; i < (rlen + 15) / 16 + 1; ++i) l[i] = 16 * i < rlen ? g[i] : uint4{0, 0, 0, 0};
        const LdsSrc src{slot};
        v = eval_walk<kReg, 0, kFeat>(c, h, src, rlen, wo, prof);
        if (v == kNeedVerify) v = eval_verify<kReg, kTier, (kFeat & kFeatDcap) != 0>(c, h, wo, &src, vm);
      } else if (inb) {
        const GlbSrc src{rw};
        v = eval_walk<kReg, 0, kFeat>(c, h, src, arena_bytes - o, wo, prof);
        if (v == kNeedVerify) v = eval_verify<kReg, kTier, (kFeat & kFeatDcap) != 0>(c, h, wo, &src, vm);
      }
      if (kTier == 1 && v == kDeferred2) {  // the large-stack tier decides it
        const uint32_t at = atomicAdd(slowq2, 1u);
        slowq2[1 + at] = ri;
        v = kDeferred;
      }
      if (v != kDeferred) verdicts[ri] = v;
    }
    if (hits) {
      const bool cnt = v != kDeferred && v < L7M_VERDICT_ALLOW_NO_PORT_POLICY;
      const uint32_t sl = v >= 0 ? static_cast<uint32_t>(v) + 2u : (v == L7M_VERDICT_DENY ? 0u : 1u);
      count_slot(hits, cnt ? sl : 0u, cnt);
    }
  }
}


template <int kHits, int kReg, int kAblate = 0, int kFeat = 0>
hipError_t launch_one(dim3 grid, size_t lds, hipStream_t stream, const uint32_t* dprog, const uint8_t* arena,
                       uint64_t arena_bytes, const uint64_t* offs, uint64_t n, int32_t* verdicts,
                       unsigned long long* hits, uint32_t stage, uint32_t* scratch = nullptr,
                       uint32_t* slowq = nullptr, DoneSignal done = DoneSignal{nullptr, nullptr, 0},
                       uint32_t* hslice = nullptr) {
  // allow > 64 KiB of dynamic LDS (gfx950: 160 KiB per CU); set per device
  // and instantiation, thread-safely (l7m_device.h)
  const hipError_t e = set_lds_attr_once(reinterpret_cast<const void*>(http_eval_kernel<kHits, kReg, kAblate, kFeat>),
                                         kHttpLdsBytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((http_eval_kernel<kHits, kReg, kAblate, kFeat>), grid, dim3(kBlock), lds, stream, dprog, arena, arena_bytes,
                     offs, n, verdicts, hits, stage, scratch, slowq, done, hslice);
  return hipGetLastError();
}

template <int kReg, int kFeat, int kTier>
hipError_t launch_slow(const HttpHeader& h, uint32_t blocks, hipStream_t stream, const uint32_t* dprog,
                              const uint8_t* arena, uint64_t arena_bytes, const uint64_t* offs, uint64_t n,
                              int32_t* verdicts, unsigned long long* hits, const uint32_t* slowq, uint32_t* slowq2,
                              uint32_t* vmscratch, uint32_t* work) {
  const size_t lds = http_slow_lds_bytes(h, kReg != 0);
  if (lds > kHttpLdsBytes) return hipErrorInvalidValue;
  const hipError_t e =
      set_lds_attr_once(reinterpret_cast<const void*>(http_slow_kernel<kReg, kFeat, kTier>), kHttpLdsBytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((http_slow_kernel<kReg, kFeat, kTier>), dim3(blocks), dim3(kSlowBlock), lds, stream, dprog, arena,
                     arena_bytes, offs, n, verdicts, hits, slowq, slowq2, vmscratch, work);
  return hipGetLastError();
}

}  // namespace
}  // namespace l7m
