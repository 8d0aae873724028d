// program.h — layout of a compiled rule set as it lives in HBM.
//
// A compiled rule set is ONE flat array of uint32 words (the "program"),
// uploaded once per device and read by the evaluation kernels through
// scalar/vector loads.  All offsets are word offsets from the start of the
// program.  The same struct definitions are used by the host compiler
// (http_compile.cc / kafka_compile.cc) and the HIP kernels.
#pragma once
#include <stdint.h>

// Host-only translation units see the HIP attributes as no-ops (HIP sources
// include hip_runtime.h before this header).
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif

namespace l7m {

constexpr uint32_t kMagicHttp = 0x3448374cu;   // "L7H4" (24-bit packed DFA + check records)
constexpr uint32_t kMagicKafka = 0x504b374cu;  // "L7KP"
constexpr uint32_t kNone = 0xffffffffu;
constexpr uint32_t kMaxFields = 64;            // present-mask is one u64 per request

// Field ids of the three pseudo headers Cilium's getHTTPRule emits
// (pkg/envoy/server.go:276-289).  Regular header fields follow.
constexpr uint32_t kFieldMethod = 0;
constexpr uint32_t kFieldPath = 1;
constexpr uint32_t kFieldAuthority = 2;

struct Span {
  uint32_t off, len;  // into the u32 pool
};

// One DFA group in packed double-array form (dfa_pack.h).  A walk starts at
// start_base and performs, per input byte b,
//     e = T[base + b];  base = (e & 0xff) == b ? e >> 8 : 0   (0 = dead)
// over the u32 slot table T (24-bit bases, byte-label ownership check).  The walk's end code is es[base]: 0 (no
// pattern), a set id (< nsets), or kLatchedAccept (0x80000000) meaning "the
// latched pattern" = latch[slot of the transition that entered the latched
// region (bases >= region)], or start_latch.  Codes are folded into one u32:
// set id, or kLatchedBit | pattern.
//
// Every table has an HBM copy in the program; the hot ones are also part of
// the LDS image (lds_* != kNone), where es/latch are stored as u16 (0xffff =
// latched accept / none).
// Skip descriptor kinds (dfa_pack.h PackedDfa::skip, DfaDesc::lds_skip).
constexpr uint32_t kSkipLoop = 1u, kSkipLit = 2u;
constexpr uint32_t kSkipMaxLit = 31, kSkipMaxPool = 512, kSkipMaxRows = 1024;

struct DfaDesc {
  uint32_t table_off;    // program: u32 T[n_slots]
  uint32_t es_off;       // program: u32 es[n_slots]
  uint32_t latch_off;    // program: u32 latch[n_slots]
  uint32_t ct_off;       // program: CandEntry ct[nsets + npats] (16 words each)
  uint32_t lds_table;    // LDS image word offset of T, or kNone
  uint32_t lds_es;       // LDS image u16 index of es16[n_slots], or kNone
  uint32_t lds_latch;    // LDS image u16 index of latch16[n_slots], or kNone
  uint32_t lds_ct;       // LDS image word offset of ct (CandEntry[]), or kNone
  uint32_t lds_mask;     // LDS image word offset of u64 pattern masks per set (npats <= 64), or kNone
  uint32_t start_base;   // 0 = dead (nothing can match)
  uint32_t region;       // bases >= region are latched (single-pattern) states
  uint32_t start_latch;  // pattern of a latched start state, else kNone
  uint32_t n_slots;
  uint32_t nsets;
  uint32_t npats;
  uint32_t set_base;     // index of this DFA's set 0 in sets[] (pattern lists)
  uint32_t field;        // field this DFA evaluates (kNone for the name DFA)
  uint32_t nstates;
  uint32_t lds_ctmask;   // LDS image word offset of a bitmask: ct entry i has candidates, or kNone
  uint32_t ctmask_off;   // program: the same bitmask (always)
  uint32_t start_es8;    // lds_es == kLdsEsInEntry: the start state's end code (es8)
  uint32_t lit_tab;      // program: u32 pairs per local pattern {word offset, length} of its
                         // literal value (kNone: not a literal), or kNone (HBM-walked DFAs only)
  uint32_t lds_skip;     // LDS image word offset of the skip descriptors (dfa_pack.h kSkip*,
                         // one word per base >= skip_lim), or kNone (LDS-walked DFAs only)
  uint32_t skip_lim;     // skip rows: bases >= skip_lim (low 16 bits); the literal pool
                         // (skip_lim >> 16 words) sits right below lds_skip
  uint32_t kind;         // kDfaPacked, or kDfaSearch (below)
  uint32_t acc_cmap_off; // kDfaSearch: program word offset of the 256-byte byte -> class map
  uint32_t acc_mid_off;  // kDfaSearch: program: u32 pattern mask per mid-set id (256)
  uint32_t acc_ncls;     // kDfaSearch: byte classes (row length of the dense table)
  uint32_t lds_search;   // kDfaSearch: LDS image word offset of the dense table (small automata), or kNone
  uint32_t lds_mid;      // kDfaSearch: LDS image word offset of its mid masks, or kNone
  uint32_t pad[2];       // 128 bytes: descriptor addresses are a shift of the DFA index
};
static_assert(sizeof(DfaDesc) == 128, "dfa desc is 32 words");

// Search automata (L7M_DIALECT_RE2_SEARCH regex fields, Go regexp
// MatchString): a dense DFA of [\x00-\xff]*(p0|...|pk), k < 32, walked as
//     e = T[state * ncls + cmap[b]];  state = e & 0xffffff;  acc |= mid[e >> 24]
// where mid[] is the mask of the patterns whose match ends at this byte with
// input left ('$' unsatisfied), and at the end acc |= es[state] (the patterns
// matching at the end of the input).  acc -- the patterns matching some
// substring -- is the walk's code: bit p = local pattern p.  start_base is the
// start state, start_es8 its mid mask; nsets is 0, so candidate entry p is
// the rules keyed on pattern p.
constexpr uint32_t kDfaPacked = 0, kDfaSearch = 1;
// kDfaAlit: a group of <= 32 literal-anchored RE2 patterns (FieldDesc::alit_*):
// no table of its own, its code (the matched-pattern mask, as for kDfaSearch)
// comes from the alit scan.
constexpr uint32_t kDfaAlit = 2;
constexpr uint32_t kSearchMaxPats = 32, kSearchMaxMid = 256;
constexpr uint32_t kLdsSearchMaxWords = 2048;  // search tables up to 8 KiB are walked from LDS

// Candidate entry of one end code (16 words): the keyed rules' check records
// (sorted by rule id) live in the check-record pool at [off, len records);
// the first record is also inlined when it has <= kCandInlineMatchers
// matchers, so the common single-candidate case costs one 64-byte read.
constexpr uint32_t kCandInlineMatchers = 4;
struct CandEntry {
  uint32_t len;       // number of check records (0 = no candidate)
  uint32_t off;       // word offset of the first record in the pool
  uint32_t rec[10];   // first record: rid, header, up to 4 x (matcher, pattern)
  uint32_t pad[4];
};
static_assert(sizeof(CandEntry) == 64, "cand entry is 16 words");
constexpr uint32_t kLatchedBit = 0x80000000u;
constexpr uint32_t kEs16Latched = 0xffffu;
// The LDS copy of a slot table names rows by image BYTE address: entry =
// 4 * (lds_table + next base) << kLdsRowShift | label, a dead transition (or
// unowned slot) = 0, i.e. row 0 = image words [0, 256), which are zero (the
// dead row shared by all tables; every read there is 0 again).  A walk step
// adds 4 * byte to the entry's upper half and reads (l7m_kernels.hip
// LdsChain).  Tables therefore end below image word kLdsTableWords (byte
// addresses fit 16 bits).
constexpr uint32_t kLdsRowShift = 16;
constexpr uint32_t kLdsTableWords = 16384;
// When a DFA has fewer than 255 end codes its LDS entries also carry the end
// code of the state they lead to: entry = row << 16 | es8 << 8 | label, es8 =
// es (0 = no match) or kEs8Latched; its lds_es is then kLdsEsInEntry and the
// walk needs no end-code table (start_es8: the start state's).
constexpr uint32_t kLdsEsInEntry = 0xfffffffeu;
constexpr uint32_t kEs8Latched = 0xffu;

// ---- HTTP kernel geometry and LDS budget -------------------------------
// Shared by the compiler's LDS image sizing (http_compile.cc) and the kernel
// (l7m_kernels.hip), so both sides agree on what the fixed part costs.
#ifndef L7M_HTTP_WAVES
#define L7M_HTTP_WAVES 16  // waves per workgroup (one workgroup per CU)
#endif
constexpr uint32_t kHttpWaves = L7M_HTTP_WAVES;
constexpr uint32_t kHttpBlock = 64 * kHttpWaves;
constexpr uint32_t kLdsBytes = 160u * 1024u;     // gfx950 LDS per CU (one workgroup)
#ifndef L7M_HTTP_WG_PER_CU
#define L7M_HTTP_WG_PER_CU 1  // resident HTTP workgroups per CU, each with its own table image
#endif
constexpr uint32_t kHttpWgPerCu = L7M_HTTP_WG_PER_CU;
constexpr uint32_t kHttpLdsBytes = kLdsBytes / kHttpWgPerCu;  // LDS of one HTTP workgroup
constexpr uint32_t kHttpRegDfas = 8;             // <= 8 value DFAs: end codes in registers
constexpr uint32_t kMaxLdsCounters = 8192;       // per-rule hit counters kept in LDS up to this
#ifndef L7M_SLICE_HITS
#define L7M_SLICE_HITS 0
#endif
// (experiment) the per-workgroup hit counters in a global slice per
// workgroup (workgroup-scope atomics in L2) instead of LDS, so the record
// stage gets their LDS
constexpr bool kSliceHits = L7M_SLICE_HITS != 0;
#ifndef L7M_SPEC_TILE
#define L7M_SPEC_TILE 1
#endif
// Batcher launches (a DoneSignal, <= 64 records, the whole batch within one
// record stage): the first wave takes every record and requests the batch's
// bytes from offset 0 before the offsets have arrived, so the two PCIe round
// trips to the pinned batch overlap, and it alone signals completion (no
// per-wave counter).  Measured (profiles/r06/ab_spec_tile_r6g.jsonl, config
// 2, 8 callers, alternated on one box): gpu phase 17.5 -> 16.1 us, 270 ->
// 293 k/s; the 64 M-request launch 4.095 -> 4.065 ms.  0: the round-5 path.
constexpr bool kSpecTile = L7M_SPEC_TILE != 0;
constexpr uint32_t kHttpMinStage = 2048;         // smallest record stage per wave (bytes)
#ifndef L7M_HTTP_MAX_STAGE
#define L7M_HTTP_MAX_STAGE 8192
#endif
constexpr uint32_t kHttpMaxStage = L7M_HTTP_MAX_STAGE;  // largest record stage per wave (bytes)
constexpr uint32_t kMaxLdsCtmaskWords = 256;     // candidate-presence bitmask kept in LDS up to this

struct FieldDesc {
  uint32_t dfa_first, ndfa;  // value DFAs of this field (contiguous)
  Span presence;             // check-record list keyed on "field present"
  // RE2-dialect gram filter (kReg = -1 programs): the field's search groups
  // are DFAs [dfa_first + search_first, dfa_first + ndfa); group j is walked
  // only when bit j % 32 of (always | the masks of the 4-byte grams the value
  // contains) is set.  gram_tab: LDS image word offset of gram_mask + 1
  // buckets of {gram, mask, gram, mask} (mask 0 = empty entry), bucket =
  // gram_bucket(gram) & gram_mask; kNone = no filter (walk every group).
  uint32_t gram_tab, gram_mask, always, search_first;
  uint32_t n_search;   // the gram filter's groups: [search_first, search_first + n_search)
  // RE2-dialect literal-anchored patterns (kDfaAlit groups, after the search
  // groups): a pattern L R (regex_ecma.h split_literal_prefix) is entered in
  // the alit table under one 4-byte gram of L at offset k; at every value
  // position q whose gram hits, L is compared at q - k and the residual
  // automaton resid_dfa (one packed DFA of the field's distinct R [\x00-\xff]*)
  // is walked from the end of L.  alit_tab: LDS image word offset of
  // alit_mask + 1 buckets {gram, rec + 1, gram, rec + 1} (0 = empty; rec =
  // the pattern's AlitRec in 16-byte granules from alit_pats), kNone = none;
  // alit_pats: word offset (16-byte aligned) of the AlitRecs -- in the LDS
  // image when alit_lds, else in the program (read once per candidate).
  uint32_t alit_tab, alit_mask, alit_pats, resid_dfa;
  uint32_t alit_lds;
  uint32_t alit_granules;  // 16-byte granules of the AlitRecs: every rec of a table entry is below it
  uint32_t dcap_mask;      // DcapSpecs (HttpHeader::lds_dcap) of this field's forced-capture patterns
};
static_assert(sizeof(FieldDesc) == 64, "field desc is 16 words");
// One literal-anchored pattern: this 16-byte header, then L's bytes zero
// padded to whole granules, so a candidate's descriptor and its first 16
// literal bytes are one 32-byte read (one round trip from the program).
struct AlitRec {
  uint32_t len_k;  // |L| | k << 16 (offset of the table gram in L)
  uint32_t code;   // kDfaAlit group DFA index << 8 | pattern bit (local id)
  uint32_t resid;  // pattern id of R in resid_dfa, or kNone: R is empty (L decides)
  uint32_t pad;
};
inline uint32_t alit_rec_granules(uint64_t lit_len) { return 1u + static_cast<uint32_t>((lit_len + 15) / 16); }
constexpr uint32_t kAlitMinPatterns = 8;          // fewer: plain search groups
// Prefilter of the alit scan: 2^14 bits right below the bucket table in the
// LDS image (FieldDesc::alit_tab - kAlitBloomWords); bit alit_bloom_bit(g) is
// set for every gram g the table holds, so a value position whose gram's bit
// is clear cannot hit the table and skips its bucket read and compares.
#ifndef L7M_ALIT_BLOOM_BITS
#define L7M_ALIT_BLOOM_BITS 0  // log2 of the prefilter's bits; 0: no prefilter (every position reads its bucket)
#endif
constexpr uint32_t kAlitBloomBits = L7M_ALIT_BLOOM_BITS;
constexpr uint32_t kAlitBloomWords = kAlitBloomBits ? (1u << kAlitBloomBits) / 32u : 0u;
__host__ __device__ inline uint32_t alit_bloom_bit(uint32_t bucket_hash) {
  return (bucket_hash >> 8) & ((1u << kAlitBloomBits) - 1u);
}
constexpr uint32_t kAlitMaxLdsBytes = 32u << 10;   // the bucket table
// Every match of a pattern contains its required literal (regex_re2.cc
// required_literals), so a value lacking all of a group's chosen 4-byte grams
// cannot match any of the group's patterns.
constexpr uint32_t kGramMinGroups = 1;      // fields with fewer search groups walk them all
constexpr uint32_t kGramMaxGroups = 64;
// (full-rate VALU only: a 24-bit multiply, no 32-bit one, which is quarter rate)
__host__ __device__ inline uint32_t gram_bucket(uint32_t gram) {
  const uint32_t x = gram ^ (gram >> 15);
  return ((x & 0xffffffu) * 0x9e3779u) >> 10;
}

// Check record (u32 words, in the check-record pool; lists are sorted by rid):
//   [0] rule id   [1] n_matchers | port entry << 8 | (has_remote_set << 31)
//   then per matcher: [field | kind << 8 | dfa << 9] [pattern]
// kind 0 = the DFA's end code must contain `pattern`, 1 = field present.
constexpr uint32_t kCrRemote = 0x80000000u;
// The rule has matchers whose automata accept a superset (back-references,
// look-ahead past its automaton limit): when its other checks pass, the
// request is decided by the slow path (regex_vm.h) -- the first pass defers
// it, http_slow_kernel evaluates it exactly.
constexpr uint32_t kCrSlow = 0x40000000u;
constexpr uint32_t kCrEntryShift = 8;
constexpr uint32_t kCrMaxMatchers = 255;
constexpr uint32_t kCrMaxEntries = 1u << 22;
__host__ __device__ inline uint32_t cr_matchers(uint32_t hd) { return hd & 0xffu; }
__host__ __device__ inline uint32_t cr_entry(uint32_t hd) { return (hd >> kCrEntryShift) & (kCrMaxEntries - 1); }

// Port entries: (endpoint policy, direction, port) -> entry id, the rule sets
// of one PortNetworkPolicy (envoy/cilium_network_policy.h:152-195).  Table of
// 2-word slots {key + 1 (0 = empty), entry | have_http << 31}.
constexpr uint32_t kEntHaveHttp = 0x80000000u;
constexpr uint32_t kMaxLdsEntWords = 1024;
__host__ __device__ inline uint32_t ent_key(uint32_t policy, uint32_t ingress, uint32_t port) {
  return policy << 17 | (ingress ? 1u : 0u) << 16 | (port & 0xffffu);
}
__host__ __device__ inline uint32_t ent_hash(uint32_t key) { return (key * 0x9e3779b1u) >> 7; }

struct HttpHeader {
  uint32_t magic;
  uint32_t n_rules;
  uint32_t n_fields;
  uint32_t n_dfas;         // value DFAs; the name DFA (if any) is dfas[n_dfas]
  uint32_t always_rule;    // smallest rule with zero matchers, or kNone
  uint32_t allow_no_l7;    // rule list empty -> L7M_VERDICT_ALLOW_NO_L7
  uint32_t has_name_dfa;
  uint32_t off_dfas;       // DfaDesc[n_dfas + has_name_dfa]
  uint32_t off_fields;     // FieldDesc[n_fields]
  uint32_t off_name_field; // u32[nsets of name DFA]: set id -> field id (kNone)
  uint32_t off_sets;       // Span[total sets]: sorted local pattern ids (into pool)
  uint32_t off_cr;         // check-record pool
  uint32_t off_pool;       // u32 pool (set pattern lists, remote ids)
  uint32_t off_remotes;    // Span[n_rules]: sorted allowed remote ids (len 0 = any)
  uint32_t any_remotes;    // 1 if no rule restricts the remote identity
  Span zero_list;          // check records of rules without matchers but with a remote set
  uint32_t lds_image_off;  // program words [off, off + words) are copied to LDS
  uint32_t lds_image_words;
  uint32_t lds_dfas;       // LDS image word offsets of the DfaDesc / FieldDesc /
  uint32_t lds_fields;     // name_field copies (always resident)
  uint32_t lds_name_field;
  uint32_t total_words;
  uint32_t lds_name_tab;   // LDS image offset of the header-name table, or kNone
  uint32_t name_tab_mask;  // its slot count - 1 (power of two)
  uint32_t single_entry;   // 1: every policy-0 request uses entry 0 (l7m_compile_http)
  uint32_t n_policies;     // endpoint policies (record policy field < n_policies)
  uint32_t ent_tab_off;    // program: port-entry table
  uint32_t lds_ent_tab;    // LDS image copy, or kNone
  uint32_t ent_mask;       // its slot count - 1
  uint32_t name_len_lo;    // bit l (l < 64, 63 = longer) set iff a referenced header
  uint32_t name_len_hi;    // name has that length: other names skip the lookup
  uint32_t cand_dfas_lo;   // bit d (n_dfas <= 64): value DFA d has candidate
  uint32_t cand_dfas_hi;   // entries for some end code (else verification skips it)
  uint32_t pres_fields_lo; // bit f: field f has a presence-keyed check-record list
  uint32_t pres_fields_hi;
  uint32_t search;         // 1: some value DFA is a kDfaSearch automaton (RE2 dialect)
  uint32_t lds_dcap;       // LDS image word offset of DcapSpec[<= kMaxDcap], or kNone
  uint32_t off_slow;       // Span[n_rules] into the pool: (field, slow program offset) pairs of the
                           // rules with kCrSlow matchers (regex_vm.h), or kNone
  uint32_t n_slow;         // rules with slow-path matchers
};
// Header-name table (LDS image): exact lower-case header names of the rules
// -> field id, open addressing on the program.h name hash; slot =
// {hash (0 = empty), len, field, image word offset of the zero-padded name}.
// Replaces the walk of the header-name DFA when it fits kMaxNameTabBytes.
constexpr uint32_t kMaxNameTabBytes = 8192;

// A back-reference pattern whose capture is forced (regex_ecma.h DcapForm,
// ECMAScript dialect): decided in the first pass.  The field's walk phase
// evaluates every DcapSpec of FieldDesc::dcap_mask on the value -- P1 compare,
// the maximal run of class bytes (length in [min, max]), L2 compare, the
// run compared with the bytes after L2, R's full-match automaton (value DFA
// rdfa, pattern 0) over the rest -- and sets bit k of the request's dcap
// mask when spec k holds.  The pattern keeps its superset automaton in the
// field's groups; a check-record matcher on it carries (k + 1) << kDcapShift
// in its pattern word, and verification requires bit k as well.
constexpr uint32_t kMaxDcap = 32;
constexpr uint32_t kDcapShift = 24;
constexpr uint32_t kPatMask = (1u << kDcapShift) - 1u;
struct DcapSpec {
  uint32_t lens;      // |P1| | |L2| << 16
  uint32_t min, max;  // run length bounds (max kNone: unbounded)
  uint32_t rdfa;      // R's automaton (a value DFA of the program), kNone: R empty (the rest must be empty)
  uint32_t cls[8];    // class bitmap: byte b in C iff bit b
  uint32_t p1;        // LDS image word offset of P1's bytes (zero-padded words)
  uint32_t l2;        // ... of L2's bytes
  uint32_t pad[2];
};
static_assert(sizeof(DcapSpec) == 64, "dcap spec is 16 words");
static_assert(sizeof(HttpHeader) == 160, "header is 40 words");

// ---------------------------------------------------------------- Kafka --
// Rule semantics follow pkg/kafka/policy.go:144-225 and
// pkg/policy/api/kafka.go:248-271 (after Sanitize, rule_validation.go:190-233).
struct KafkaRuleDesc {
  uint32_t flags;       // kKRule* bits
  int32_t version;      // apiVersionInt when kKRuleVersion
  uint32_t keys_lo;     // apiKeyInt as a bitmask over kinds 0..63 (unless kKRuleAnyKey)
  uint32_t keys_hi;
  uint32_t client_idx;  // interned ClientID when kKRuleClient (KafkaClientSlot::idx)
  uint32_t group;       // L7DataMap entry (bit of the source's selector mask)
  uint32_t pad[2];
};
constexpr uint32_t kKRuleAnyKey = 1u, kKRuleVersion = 2u, kKRuleTopic = 4u, kKRuleClient = 8u;

// Open-addressed (linear probing) table: Topic -> ascending ids of the rules
// whose Topic equals it.  hash == 0 marks an empty slot (see name_hash_final).
// One 32-byte slot carries the check fields of the topic's first rule and
// the first kTopicInline bytes of the topic (zero padded), so the common
// case (short names, first rule decides) resolves with one slot fetch; the
// rest lives in the parallel KafkaTopicExt array.
constexpr uint32_t kTopicInline = 16;
struct KafkaTopicSlot {
  uint32_t hash;
  uint32_t meta;       // len (8) | kset (6) << 8 | version-cond << 14 | client-cond << 15 | (u16)version << 16
  uint32_t r0;         // first rule id | (more than one rule) << 31
  uint32_t r0_client;  // its client_idx (low 16 bits, 0xffff = none) | its group << 16
  uint32_t pfx[kTopicInline / 4];
};
struct KafkaTopicExt {
  uint32_t str_off;  // whole topic in the string area
  Span rules;        // ascending rule ids in the u32 pool
  uint32_t pad;
};
constexpr uint32_t kSlotVersionCond = 1u << 14, kSlotClientCond = 1u << 15, kSlotMore = 1u << 31;
// Rule topics are at most 255 bytes (Sanitize, rule_validation.go:222-226).
constexpr uint32_t kMaxTopicLen = 255;
// Distinct apiKey sets ("ksets"): id 0 = any kind; the kind_ok table holds,
// per request kind (0..63, 64 = other), a bit per kset id that accepts it.
constexpr uint32_t kMaxKsets = 64;

// Interned rule ClientIDs: one lookup per request turns its ClientID into
// the index a rule's client_idx is compared with.
constexpr uint32_t kClientInline = 16;
struct KafkaClientSlot {
  uint32_t hash;
  uint32_t str_len;
  uint32_t str_off;
  uint32_t idx;
  uint32_t pfx[kClientInline / 4];
};

constexpr uint32_t kKafkaKinds = 65;  // request kinds 0..63; [64] = any other value

struct KafkaHeader {
  uint32_t magic;
  uint32_t n_rules;
  uint32_t off_rules;    // KafkaRuleDesc[n_rules]
  uint32_t off_slots;    // KafkaTopicSlot[n_slots]
  uint32_t n_slots;      // power of two (0 when no rule has a Topic)
  uint32_t off_pool;     // u32 pool
  uint32_t off_crc;      // u32[256] CRC-32 (IEEE) table for message-set CRCs
  uint32_t off_strings;  // byte area (word offset)
  uint32_t total_words;
  uint32_t off_clients;  // KafkaClientSlot[n_clients]
  uint32_t n_clients;    // power of two (0 when no rule has a ClientID)
  uint32_t off_ext;      // KafkaTopicExt[n_slots]
  uint32_t off_kind_ok;  // u64[kKafkaKinds]
  uint32_t off_ids;      // KafkaIdSlot[1 + n_id_slots]: [0] = the wildcard entries' mask
  uint32_t n_id_slots;   // power of two; 0 = one wildcard entry (every rule applies)
  uint32_t pad;
  // Ascending ids of the rules whose CheckAPIKeyRole(kind) holds:
  Span notopic_by_kind[kKafkaKinds];  // ... and Topic == ""
  Span all_by_kind[kKafkaKinds];      // ... any Topic
};
// Source identity -> mask of the L7DataMap entries whose rules apply to it
// (the selecting entries' bits | the wildcard entries' bits); open
// addressing on kafka_id_hash, identity 0 = empty.
struct KafkaIdSlot {
  uint32_t identity;
  uint32_t pad;
  uint32_t mask_lo, mask_hi;
};
constexpr uint32_t kMaxKafkaGroups = 64;
__host__ __device__ inline uint32_t kafka_id_hash(uint32_t id) {
  id ^= id >> 16;
  id *= 0x7feb352du;
  id ^= id >> 15;
  id *= 0x846ca68bu;
  return id ^ (id >> 16);
}
static_assert(sizeof(KafkaRuleDesc) == 32, "rule desc is 8 words");
static_assert(sizeof(KafkaTopicSlot) == 32, "topic slot is 8 words");
static_assert(sizeof(KafkaTopicExt) == 16, "topic ext is 4 words");
static_assert(sizeof(KafkaClientSlot) == 32, "client slot is 8 words");
static_assert(sizeof(KafkaHeader) % 16 == 0, "header is whole 16-byte lines");

// Key hash of the Kafka topic / ClientID tables and the HTTP header-name
// table: the name as ceil(len / 4) little-endian u32 words (the last one zero
// padded), each folded in by a step of full-rate VALU operations (xor, a 24-bit
// multiply-add, a rotate: no quarter-rate 32-bit multiply per word), then a
// murmur3 finalizer over the length; 0 is remapped (0 marks an empty slot).
// Device code hashes the first kNameHashMinWords words from registers it
// already holds for the compare, word-wise without byte extraction.
constexpr uint32_t kNameHashMinWords = 6;
__host__ __device__ inline uint32_t name_hash_step(uint32_t h, uint32_t w) {
  const uint32_t x = h ^ w;
  return (x & 0xffffffu) * 0x9e3779u + ((x << 13) | (x >> 19));
}
__host__ __device__ inline uint32_t name_hash_final(uint32_t h, uint32_t len) {
  h = (h ^ len) * 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h ? h : 1u;
}

// isTopicAPIKey (pkg/kafka/policy.go:27-52) as a mask over kinds 0..63.
constexpr uint64_t kTopicApiKeyMask =
    (1ull << 0) | (1ull << 1) | (1ull << 2) | (1ull << 3) | (1ull << 4) | (1ull << 5) |
    (1ull << 6) | (1ull << 8) | (1ull << 9) | (1ull << 19) | (1ull << 20) | (1ull << 21) |
    (1ull << 23) | (1ull << 24) | (1ull << 27) | (1ull << 28) | (1ull << 34) | (1ull << 35) |
    (1ull << 37);

// optiopay/kafka maxParseBufSize (vendor/github.com/optiopay/kafka/proto/utils.go:9).
constexpr int64_t kKafkaMaxParseBuf = 100LL * 65535;

}  // namespace l7m
