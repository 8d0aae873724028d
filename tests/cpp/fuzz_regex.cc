// Differential fuzzer: libl7match's ECMAScript parser + DFA builders (the
// plain subset construction, the context / obligation construction for \b,
// \B and look-ahead, and the packed field automaton of dfa_pack.h) versus
// libstdc++ std::regex_match (the engine Envoy applies to HeaderMatcher
// regexes, envoy/cilium_network_policy.h:68-71).  Patterns with
// back-references are determinised as a superset (lower_for_dfa): the DFA
// must accept everything std::regex accepts.  Test infrastructure only.
//   fuzz_regex <seed> <n_patterns> <strings_per_pattern> [assertions 0/1]
#include <cstdio>
#include <cstdlib>
#include <random>
#include <regex>
#include <string>
#include <vector>

#include "../../cilium_amd/csrc/dfa_pack.h"
#include "../../cilium_amd/csrc/regex_ecma.h"
#include "../../cilium_amd/csrc/regex_vm.h"

using namespace l7m::re;
static std::mt19937_64 rng;
static int rnd(int n) { return (int)(rng() % (uint64_t)n); }
static bool g_assert = false;  // generate \b \B (?=) (?!) and back-references
static int g_groups = 0;       // capture groups opened so far in the pattern being generated

static const char* kAtoms[] = {"a", "b", "c", "x", ".", "\\d", "\\w", "\\s", "\\D", "\\W", "\\S",
  "[ab]", "[^a]", "[a-c]", "[]", "[^]", "[\\d-]", "[-a]", "[a-]", "\\.", "/", "-", "_", "0", "9",
  "[[:alpha:]]", "[[:digit:]x]", "[^[:space:]]", "\\x41", "\\u0062", "\\cA", "\\k", "\\/", "[\\]a]",
  "[[=a=]]", "[[.b.]]", "\\t", "[\\x80-\\xff]", "[A-z]", "[\\W\\d]", "\\0", "}", "]", "A", "Z"};

// Nested quantifiers are rationed: libstdc++'s backtracking executor is
// exponential on them (the reference's own catastrophic case).
static std::string gen(int depth, bool* quant) {
  int k = rnd(depth > 3 ? 3 : 10);
  std::string s;
  bool q1 = false, q2 = false, q3 = false;
  if (k < 4) s = kAtoms[rnd(sizeof(kAtoms) / sizeof(*kAtoms))];
  else if (k < 6) s = gen(depth + 1, &q1) + gen(depth + 1, &q2);
  else if (k < 7) s = gen(depth + 1, &q1) + "|" + gen(depth + 1, &q2);
  else if (k < 8) {
    ++g_groups;
    s = "(" + gen(depth + 1, &q1) + ")";
  }
  else if (k < 9) s = "(?:" + gen(depth + 1, &q1) + ")";
  else s = gen(depth + 1, &q1) + gen(depth + 1, &q2) + gen(depth + 1, &q3);
  *quant = q1 || q2 || q3;
  int q = *quant ? rnd(10) : rnd(12);  // stacked forms only on quantifier-free bodies
  static const char* qs[] = {"*", "+", "?", "{2}", "{0,2}", "{1,}", "*?", "+?", "??", "{0}", "**", "{1}{2}"};
  if (rnd(3) == 0 && (!*quant || rnd(40) == 0)) {
    s = "(?:" + s + ")" + qs[q];
    *quant = true;
  }
  if (rnd(20) == 0) s = "^" + s;
  if (rnd(20) == 0) s = s + "$";
  if (g_assert) {
    if (rnd(6) == 0) s = (rnd(2) ? "\\b" : "\\B") + s;
    if (rnd(6) == 0) s = s + (rnd(2) ? "\\b" : "\\B");
    if (rnd(8) == 0) {
      bool ql = false;
      s = (rnd(2) ? "(?=" : "(?!") + gen(depth + 2, &ql) + ")" + s;
    }
    if (g_groups && rnd(10) == 0) s = s + "\\" + std::to_string(1 + rnd(g_groups));
  }
  return s;
}

static std::string rand_input() {
  static const char alpha[] = "abcxABZ09_ -./\t\n\r]}aab";
  int n = rnd(8);
  std::string s;
  for (int i = 0; i < n; ++i) {
    if (rnd(16) == 0) s.push_back((char)rnd(256));
    else s.push_back(alpha[rnd(sizeof(alpha) - 1)]);
  }
  return s;
}

static bool dfa_match(const Dfa& d, const std::string& s, uint32_t pat) {
  uint32_t st = d.start;
  for (unsigned char c : s) st = d.next[st * d.ncls + d.cmap[c]];
  const auto& set = d.sets[d.endset[st]];
  for (uint32_t p : set) if (p == pat) return true;
  return false;
}

int main(int argc, char** argv) {
  rng.seed(argc > 1 ? strtoull(argv[1], 0, 10) : 1);
  int npat = argc > 2 ? atoi(argv[2]) : 2000;
  int nstr = argc > 3 ? atoi(argv[3]) : 200;
  g_assert = argc > 4 && atoi(argv[4]) != 0;
  long checked = 0, mism = 0, unsup = 0, rejected = 0, parse_mism = 0, superset = 0, packed_mism = 0;
  long vm_checked = 0, vm_mism = 0, vm_limit = 0;
  long accept_mism = 0;
  std::vector<uint32_t> scratch(1u << 16);
  // fixed cases: references to a group that is still open are error_backref
  // in libstdc++ (_M_insert_backref); chained references must lower in bounded
  // size (each level doubles a literal copy)
  {
    std::string chain = "(a)";
    for (int k = 1; k < 40; ++k) chain += "(\\" + std::to_string(k) + "\\" + std::to_string(k) + ")";
    const char* fixed[] = {"(a\\1)", "(a(b\\2))", "(x(y|\\2))", "((a)\\1)", "(a)\\1", "(a)(b\\1)"};
    for (const char* fp : fixed) {
      bool sok = true;
      try { std::regex r(fp, std::regex::ECMAScript); } catch (...) { sok = false; }
      Ast fa; std::string ferr;
      const bool pok = parse_ecma(fp, &fa, &ferr) == Status::Ok;
      if (sok != pok) { ++accept_mism; printf("FIXED-MISMATCH %s std=%d ours=%d\n", fp, sok, pok); }
    }
    Ast ca; std::string cerr;
    if (parse_ecma(chain, &ca, &cerr) != Status::Ok) { ++accept_mism; printf("CHAIN-PARSE %s\n", cerr.c_str()); }
    bool cex = true;
    Ast cl = lower_for_dfa(ca, &cex);
    if (cex || cl.nodes.size() > (1u << 16)) { ++accept_mism; printf("CHAIN-LOWER nodes=%zu\n", cl.nodes.size()); }
  }
  for (int i = 0; i < npat; ++i) {
    bool qq = false;
    g_groups = 0;
    std::string p = gen(0, &qq);
    if (getenv("FUZZ_TRACE")) { fprintf(stderr, "P %d %s\n", i, p.c_str()); }
    std::regex r;
    bool ok = true;
    try { r = std::regex(p, std::regex::ECMAScript | std::regex::optimize); } catch (...) { ok = false; }
    Ast full; std::string err;
    Status st = parse_ecma(p, &full, &err);
    if (!ok) {
      rejected++;
      if (st == Status::Ok) {  // std::regex rejects what the parser accepted
        ++accept_mism;
        if (accept_mism < 20) printf("ACCEPT-MISMATCH %s\n", p.c_str());
      }
      continue;
    }
    if (st == Status::Unsupported) { unsup++; continue; }
    if (st != Status::Ok) { parse_mism++; printf("PARSE-MISMATCH %s : %s\n", p.c_str(), err.c_str()); continue; }
    // the slow path (libstdc++'s executor restated) must equal std::regex on
    // every pattern, back-references included
    std::vector<uint32_t> vprog;
    std::string verr;
    const bool have_vm = l7m::vm_compile(full, &vprog, &verr);
    bool exact = true;
    Ast a = lower_for_dfa(full, &exact);
    if (!exact) superset++;
    // Two-pattern DFA (pattern + a literal) also exercises multi-pattern sets.
    Ast lit = literal_ast("ab");
    Dfa d; DfaLimits lim;
    lim.max_states = 1u << 16;
    if (build_dfa({&a, &lit}, lim, &d) != Status::Ok) { unsup++; continue; }
    // the packed field automaton (literal-prefix split, residual product)
    l7m::PackedDfa pk;
    const bool have_pk = l7m::build_field_dfa({&a, &lit}, l7m::FieldDfaLimits(), &pk) == Status::Ok;
    std::vector<std::string> ins;
    for (int j = 0; j < nstr; ++j) ins.push_back(rand_input());
    ins.push_back(""); ins.push_back("ab");
    for (const auto& s : ins) {
      bool ref = std::regex_match(s, r);
      if (have_vm) {
        const int v = l7m::vm_match(vprog.data(), reinterpret_cast<const uint8_t*>(s.data()),
                                    static_cast<uint32_t>(s.size()), scratch.data(),
                                    static_cast<uint32_t>(scratch.size()), 1u << 22);
        ++vm_checked;
        if (v == l7m::kVmLimit) ++vm_limit;
        else if ((v == l7m::kVmMatched) != ref) {
          ++vm_mism;
          if (vm_mism < 20) {
            printf("VM-MISMATCH pat=%s in=", p.c_str());
            for (unsigned char ch : s) printf("\\x%02x", ch);
            printf(" ref=%d vm=%d\n", ref, v);
          }
        }
      }
      bool got = dfa_match(d, s, 0);
      bool gotlit = dfa_match(d, s, 1);
      checked++;
      if (have_pk) {
        const uint32_t code = l7m::packed_walk(pk, reinterpret_cast<const uint8_t*>(s.data()), s.size());
        bool pk0 = false;
        if (code & l7m::kLatchedAccept) pk0 = (code & ~l7m::kLatchedAccept) == 0;
        else for (uint32_t q : pk.sets[code]) pk0 |= q == 0;
        if (pk0 != got) {
          packed_mism++;
          if (packed_mism < 10) printf("PACKED-MISMATCH pat=%s dfa=%d packed=%d\n", p.c_str(), got, pk0);
        }
      }
      if (!exact) {  // superset automaton: every std::regex match must be accepted
        if (ref && !got) {
          mism++;
          if (mism < 30) printf("SUPERSET-MISS pat=%s\n", p.c_str());
        }
        continue;
      }
      if (ref != got || gotlit != (s == "ab")) {
        mism++;
        if (mism < 30) {
          printf("MISMATCH pat=%s in=", p.c_str());
          for (unsigned char c : s) printf("\\x%02x", c);
          printf(" ref=%d got=%d\n", ref, got);
        }
      }
    }
  }
  printf("checked=%ld mismatches=%ld unsupported=%ld rejected_by_std=%ld parse_mismatch=%ld superset=%ld "
         "packed_mismatch=%ld vm_checked=%ld vm_mismatch=%ld vm_limit=%ld accept_mismatch=%ld\n", checked, mism, unsup,
         rejected, parse_mism, superset, packed_mism, vm_checked, vm_mism, vm_limit, accept_mism);
  return (mism || parse_mism || packed_mism || vm_mism || vm_limit || accept_mism) ? 1 : 0;
}
