// dfa_pack.h — pack a multi-pattern DFA into the GPU's byte-indexed
// double-array form ("DA table") with single-pattern tail sharing.
//
// Why: a dense (states x classes) table for 1k realistic rules is megabytes
// (every pattern owns a private copy of shared tails such as
// `/v[0-9]+/(users|orders|items)/[0-9]+`, and trie-like prefix states are
// almost all dead entries), so every DFA step would be a random L2 access.
// The packed form below is 10-100x smaller and usually fits gfx950's LDS,
// and a step is ONE dependent 4-byte LDS read indexed by the raw input byte
// (no byte-class lookup on the critical path):
//
//     e = T[base + byte];
//     base = (e & 0xffff) == base ? e >> 16 : 0;     // base 0 = dead state
//
// Every non-dead transition is an explicit slot whose check half holds the
// owner's base; a slot another state owns (or an empty one, check 0xffff)
// means "dead".  The dead state owns no slot, so it is absorbing.
//
// Tail sharing ("latching"): a state from which exactly one pattern can still
// match is "latched".  Latched states are minimised with binary acceptance,
// so all patterns whose residual languages coincide share ONE copy of the
// tail; the pattern identity is recovered from the slot of the transition
// that entered the latched region (LATCH[slot]), or from start_latch when the
// start state itself is latched.  All latched states have base >= region.
#pragma once
#include <cstdint>
#include <vector>

#include "regex_ecma.h"

namespace l7m {

constexpr uint32_t kLatchedAccept = 0x80000000u;  // end code: accept the latched pattern
constexpr uint32_t kMaxDaBase = 65535 - 256;      // 16-bit bases and slots

struct PackedDfa {
  uint32_t n_slots = 0;          // table length incl. 256 slots of tail padding
  std::vector<uint32_t> table;   // check | next_base << 16; empty slot check = 0xffff
  std::vector<uint32_t> es;      // per base: 0 no match, set id (index into sets), or kLatchedAccept
  std::vector<uint32_t> latch;   // per slot: pattern entered by that transition (0xffffffff none)
  uint32_t start_base = 0;       // 0 = dead start (nothing can match)
  uint32_t region = 1;           // bases >= region are latched states
  uint32_t start_latch = 0xffffffffu;
  uint32_t nstates = 0;          // packed states incl. dead
  uint32_t n_explicit = 0;       // explicit transitions
  std::vector<std::vector<uint32_t>> sets;  // end sets (set id -> sorted pattern ids), set 0 empty
};

// Returns Ok, or TooBig when a slot would exceed 16 bits (caller splits).
re::Status pack_dfa(const re::Dfa& d, PackedDfa* out);

// Reference walk of a packed DFA on the host (tests / interpreter parity):
// returns the end code (0, set id, or kLatchedAccept | pattern).
uint32_t packed_walk(const PackedDfa& p, const uint8_t* s, size_t n);

}  // namespace l7m
