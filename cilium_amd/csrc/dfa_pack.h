// dfa_pack.h — the GPU's packed multi-pattern automaton ("DA table") and the
// scalable builder that produces it for one header field.
//
// Packed form (one u32 slot table T per field automaton):
//
//     e = T[base + byte];
//     base = (e & 0xff) == byte ? e >> 8 : 0;          // base 0 = dead state
//
// Every non-dead transition is an explicit slot holding the target's base
// (24 bits) and the input byte it was placed for (8 bits).  Bases are unique
// per state, so slot s can only be "base + byte" for the state whose base is
// s - label: the byte label is a complete ownership check (no owner field).
// An empty slot is 0 (next base 0 = dead whatever its label).  One step is
// ONE dependent 4-byte read indexed by the raw input byte; 24-bit bases
// address 16 M slots, so a whole field (100k rules) is one automaton.
//
// Tail sharing ("latching"): a state from which exactly one pattern can still
// match is "latched".  Latched states are the residual automata of the
// patterns, shared by every pattern with the same residual (config 2: the
// 500 `/svc{i}/v[0-9]+/(users|orders|items)/[0-9]+` rules share one tail;
// config 5: the 20k `(.{0,8}){1,8}foo` rules share one), so the pattern
// identity is recovered from the slot of the transition that entered the
// latched region (latch[slot]) or from start_latch when the start state itself
// is latched.  All latched states have base >= region.
//
// Builder (build_field_dfa): each pattern is split into a literal prefix and a
// residual regex; distinct residuals are determinised once (regex_ecma.h
// build_dfa); the multi-pattern part is the product of the per-pattern DFAs
// over a field-wide byte partition, computed only until a single pattern
// remains live (for literal-prefixed rule sets it is the prefix trie).  Cost
// is linear in the rules for prefix-diverging sets instead of a subset
// construction over the union NFA.
#pragma once
#include <cstdint>
#include <vector>

#include "program.h"
#include "regex_ecma.h"

namespace l7m {

constexpr uint32_t kLatchedAccept = 0x80000000u;  // end code: accept the latched pattern
constexpr uint32_t kMaxDaBase = (1u << 24) - 1 - 256;  // 24-bit bases and slots

struct PackedDfa {
  uint32_t n_slots = 0;          // table length incl. 256 slots of tail padding
  std::vector<uint32_t> table;   // next_base << 8 | byte label; empty slot 0
  std::vector<uint32_t> es;      // per base: 0 no match, set id (index into sets), or kLatchedAccept
  std::vector<uint32_t> latch;   // per slot < region + 256: pattern entered by that transition (0xffffffff none)
  uint32_t start_base = 0;       // 0 = dead start (nothing can match)
  uint32_t region = 1;           // bases >= region are latched states
  uint32_t start_latch = 0xffffffffu;
  uint32_t nstates = 0;          // packed states incl. dead
  uint64_t n_explicit = 0;       // explicit transitions
  uint32_t n_multi = 0;          // multi-pattern (product) states
  uint32_t n_residuals = 0;      // distinct residual automata
  std::vector<std::vector<uint32_t>> sets;  // end sets (set id -> sorted pattern ids), set 0 empty
  // Skip descriptors of latched rows (the walk's fast paths, see skip_kind):
  // every row with base >= skip_lim has one, skip[base - skip_lim]; 0 = none.
  uint32_t skip_lim = 0;              // 0: no skip rows
  std::vector<uint32_t> skip;         // per base in [skip_lim, max base]
  std::vector<uint8_t> skip_lits;     // literal pool of kSkipLit rows
};

// Skip descriptor word (latched rows only, so slast is unaffected):
//   kSkipLoop: every transition of the row returns to the row itself: the
//     rest of the field stays in the row iff each byte b has T[base + b]
//     labelled b (independent lookups), else the walk is dead.
//   kSkipLit:  the row starts a run of n >= 2 non-accepting single-transition
//     rows (a literal): the next n bytes must equal skip_lits[off, off + n)
//     (else dead; a field ending inside the run does not match either), and
//     the walk continues from the entry T[tslot] (the run's last transition).
//   word = kind | n << 2 | off << 7 | tslot << 16   (n <= 31, off < 512, tslot < 64 Ki)
// (kSkipLoop / kSkipLit and the limits are in program.h, shared with the kernels)

struct FieldDfaLimits {
  size_t max_multi_states = 1u << 21;  // product states before the caller splits the pattern set
  uint64_t max_slots = kMaxDaBase;     // packed bases
};

// Build the packed automaton of patterns[0..n) (pattern id = index).
// Returns Ok, TooBig (a limit was exceeded: the caller splits the set) or
// the first residual's build_dfa error.
re::Status build_field_dfa(const std::vector<const re::Ast*>& patterns, const FieldDfaLimits& lim,
                           PackedDfa* out);

// Reference walk of a packed DFA on the host (tests / interpreter parity):
// returns the end code (0, set id, or kLatchedAccept | pattern).
uint32_t packed_walk(const PackedDfa& p, const uint8_t* s, size_t n);

// Explicit-transition estimate of one pattern (its literal prefix plus its
// residual automaton), used to chunk huge pattern sets before building.
uint64_t pattern_slot_estimate(const re::Ast& a);

}  // namespace l7m
