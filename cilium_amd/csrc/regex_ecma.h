// regex_ecma.h — ECMAScript (libstdc++ std::regex dialect) parser and the
// multi-pattern DFA builder used to compile Cilium L7 HTTP rules.
//
// Reference semantics: Envoy's HeaderData builds `std::regex(value,
// std::regex::optimize)` (ECMAScript grammar) and matches with
// `std::regex_match` (full match) — see the vendored HeaderMatcher docs
// pkg/envoy/envoy/api/v2/route/route.pb.go:2420-2430 and the call site
// envoy/cilium_network_policy.h:68-71.  This file restates the libstdc++
// ECMAScript grammar (scanner/compiler of GCC 11) as an AST, lowers it to a
// Thompson NFA and determinises a *set* of patterns into one DFA whose end
// column reports which patterns matched.  No backtracking, no recursion on the
// input.  Word boundaries (\b / \B) and look-ahead ((?=X) / (?!X)) are
// regular and determinised exactly (build_dfa's context / obligation
// construction); back-references are not regular: lower_for_dfa replaces them
// (and any look-ahead past the DFA limits) by a superset and marks the
// pattern for the exact slow path (regex_vm.h), which restates libstdc++'s
// backtracking executor.
#pragma once
#include <bitset>
#include <cstdint>
#include <string>
#include <vector>

namespace l7m {
namespace re {

using ByteSet = std::bitset<256>;

enum class Status { Ok = 0, Syntax = 1, Unsupported = 2, TooBig = 3 };

struct Node {
  // Group / Backref appear only in parse_ecma's full AST (lower_for_dfa
  // removes them); WordB / Look are determinised by build_dfa.
  enum Kind : uint8_t { Empty, Set, Cat, Alt, Rep, Bol, Eol, WordB, Look, Group, Backref } kind = Empty;
  ByteSet set;            // Set
  std::vector<int> kids;  // Cat / Alt / Rep(1) / Look(1: the looked-ahead pattern) / Group(1)
  int min = 0, max = 0;   // Rep: repeat bounds, max < 0 = unbounded
                          // WordB / Look: min = 1 for the negated form (\B, (?!X))
                          // Group / Backref: min = capture index (1-based)
  bool lazy = false;      // Rep: non-greedy ('?' after the quantifier; exploration order only)
  bool brace = false;     // Rep: written {n}, {n,} or {n,m} (libstdc++ builds those from copies)
};

struct Ast {
  std::vector<Node> nodes;
  int root = -1;
};

// Parse `pat` with the libstdc++ ECMAScript grammar into the full AST (capture
// groups, back-references, word boundaries, look-ahead).  Patterns that
// std::regex rejects are expected to be filtered by the caller first (the
// compiler validates with std::regex itself); this parser reports Syntax for
// anything it cannot parse.
Status parse_ecma(const std::string& pat, Ast* out, std::string* err);

// The AST build_dfa determinises: capture groups dissolved, every
// back-reference \k replaced by a copy of group k's pattern (a superset: the
// referenced text is a string that group matched).  *exact = false when a
// back-reference was replaced (the DFA's answer is then a superset and the
// pattern needs the slow path).
Ast lower_for_dfa(const Ast& a, bool* exact);
// Look-ahead replaced by the empty pattern (a superset), for patterns whose
// exact automaton exceeds the limits.
Ast drop_lookahead(const Ast& a);
bool has_node(const Ast& a, Node::Kind k);

// Parse `pat` as Go regexp (RE2) syntax for L7M_DIALECT_RE2_SEARCH
// (regex_re2.cc): Syntax where regexp.Compile fails, Unsupported for valid
// RE2 outside the byte-exact subset.
Status parse_re2(const std::string& pat, Ast* out, std::string* err);

// Wrap a parsed pattern for unanchored search (regexp.MatchString):
// [\x00-\xff]* p [\x00-\xff]*.
void make_search(Ast* a);

// AST matching exactly the bytes of `lit` (Envoy HeaderMatchType::Value).
Ast literal_ast(const std::string& lit);

// One compiled DFA over a set of patterns.
struct Dfa {
  int ncls = 0;                 // byte classes
  uint8_t cmap[256] = {0};      // byte -> class
  int nstates = 0;              // state 0 is the dead state
  int start = 0;
  std::vector<uint32_t> next;   // nstates * ncls, next-state ids
  std::vector<uint32_t> endset; // nstates: id into sets (0 = empty set)
  std::vector<uint32_t> midset; // nstates (build_dfa with_mid only): patterns matched here
                                // when the input does NOT end here ('$' not satisfied)
  std::vector<std::vector<uint32_t>> sets;  // set id -> sorted pattern ids
};

struct DfaLimits {
  size_t max_states = 1u << 20;
  size_t max_table_bytes = 64ull << 20;  // (ncls + 1) * 4 * states
};

// Determinise patterns[0..n) (pattern id = index) into one minimised DFA with
// states numbered breadth-first from the start state.  Returns TooBig when a
// limit is exceeded (caller splits the pattern set).
Status build_dfa(const std::vector<const Ast*>& patterns, const DfaLimits& lim, Dfa* out, bool with_mid = false);

// Prefix a pattern with [\x00-\xff]* (a match may start anywhere): with
// build_dfa's mid sets, the patterns matching a substring that ends at each
// position of the input (regexp.MatchString = the union over positions).
void make_search_prefix(Ast* a);

// Cut a search pattern's trailing repetitions to their minimum (equivalent
// under regexp.MatchString, regex_re2.cc).
void simplify_search(Ast* a);

// Byte strings every match of the pattern contains (regex_re2.cc): the
// literal runs of its top-level structure.  Empty when nothing is required.
std::vector<std::string> required_literals(const Ast& a);

// RE2 search patterns of the form L R (regex_re2.cc): L the literal prefix
// (>= 4 bytes) of the top-level concatenation, R the rest, with no ^, \b or
// look-around in R.  Under MatchString such a pattern matches iff some
// occurrence of L in the value is followed by bytes that start with a match
// of R; *resid = R [\x00-\xff]* (its full-match automaton answers that).
bool split_literal_prefix(const Ast& a, std::string* lit, Ast* resid);
bool residual_is_empty(const Ast& resid);  // R was empty: L alone decides
std::string ast_key(const Ast& a);          // structural key (dedupes residuals)

// Back-references whose capture is forced (ECMAScript full match).  A pattern
//     [^] P1 ( C{n,m} ) L2 \k R
// -- P1 and L2 literal byte strings, C one byte class, the first byte of L2
// outside C, k the pattern's only back-reference, R regular with no ^, \b,
// \B or look-ahead -- matches a value v iff v starts with P1, the maximal run
// of C bytes after it has a length r in [n, m], L2 follows it, the same r
// bytes follow L2, and R full-matches the rest: group k cannot end anywhere
// but at the first byte outside C (L2[0] must follow it), so the capture is
// that run and no backtracking can choose another.  E.g. /(\w+)/\1(/.*)?
// (P1 "/", C \w, L2 "/", R (/.*)?).  Such patterns are decided in the first
// pass by byte compares (program.h DcapSpec) instead of the slow path.
struct DcapForm {
  std::string p1, l2;
  ByteSet cls;
  int min = 1, max = -1;  // max < 0: unbounded
  bool r_empty = true;
  Ast r;                  // R, lowered (groups dissolved); full-match automaton
};
bool analyze_dcap(const Ast& full, DcapForm* out);

}  // namespace re

// The slow path's program for a full AST (regex_vm.cc, executed by
// regex_vm.h vm_match); false (with *err) past its size limit.
bool vm_compile(const re::Ast& full, std::vector<uint32_t>* out, std::string* err);

}  // namespace l7m
