// Differential fuzzer: the oracle's Thompson-NFA / Pike-VM simulator
// (oracle/nfa.h) versus libstdc++ std::regex (the engine Envoy applies to
// HeaderMatcher regexes, envoy/cilium_network_policy.h:68-71).  Test
// infrastructure only.
//   fuzz_nfa <seed> <n_patterns> <strings_per_pattern> <n_long>
// Three regimes:
//   1. random grammar patterns x short random subjects: regex_match vs full,
//      regex_search vs search;
//   2. noisy pattern strings: std::regex throws <=> the NFA parser throws;
//   3. subjects of 1 - 8 KiB on pattern families std::regex evaluates without
//      catastrophic backtracking (its stack is fine below ~10 KB).
// Prints "checked N mismatches M rejected R unsupported U" and the first few
// mismatches; exit status 1 on any mismatch.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <regex>
#include <string>
#include <vector>

#include "../../oracle/nfa.h"

static std::mt19937_64 rng;
static int rnd(int n) { return (int)(rng() % (uint64_t)n); }

static const char* kAtoms[] = {"a", "b", "c", "x", ".", "\\d", "\\w", "\\s", "\\D", "\\W", "\\S",
  "[ab]", "[^a]", "[a-c]", "[]", "[^]", "[\\d-]", "[-a]", "[a-]", "\\.", "/", "-", "_", "0", "9",
  "[[:alpha:]]", "[[:digit:]x]", "[^[:space:]]", "\\x41", "\\u0062", "\\cA", "\\k", "\\/", "[\\]a]",
  "[[=a=]]", "[[.b.]]", "\\t", "[\\x80-\\xff]", "[A-z]", "[\\W\\d]", "\\0", "}", "]", "A", "Z",
  "[a-c-e]", "[--/]", "[\\b]", "[^\\D]", "[[:upper:][:digit:]]", "\\b", "\\B", "[\\s\\S]", "[.]"};

static std::string gen(int depth, bool* quant) {
  int k = rnd(depth > 3 ? 3 : 10);
  std::string s;
  bool q1 = false, q2 = false, q3 = false;
  if (k < 4) s = kAtoms[rnd(sizeof(kAtoms) / sizeof(*kAtoms))];
  else if (k < 6) s = gen(depth + 1, &q1) + gen(depth + 1, &q2);
  else if (k < 7) s = gen(depth + 1, &q1) + "|" + gen(depth + 1, &q2);
  else if (k < 8) s = "(" + gen(depth + 1, &q1) + ")";
  else if (k < 9) s = "(?:" + gen(depth + 1, &q1) + ")";
  else s = gen(depth + 1, &q1) + gen(depth + 1, &q2) + gen(depth + 1, &q3);
  *quant = q1 || q2 || q3;
  static const char* qs[] = {"*", "+", "?", "{2}", "{0,2}", "{1,}", "*?", "+?", "??", "{0}", "**", "{1}{2}", "{1,3}?"};
  // stacked forms ("**", "{1}{2}") nest quantifiers: single atoms only
  int q = k < 4 ? rnd(13) : rnd(10);
  if (q >= 10 && q != 12 && k >= 4) q = 0;
  if (rnd(3) == 0 && !*quant) {  // no random nesting: the backtracker is exponential on it
    s = "(?:" + s + ")" + qs[q];
    *quant = true;
  }
  if (rnd(20) == 0) s = "^" + s;
  if (rnd(20) == 0) s = s + "$";
  return s;
}

static std::string rand_input(int maxlen) {
  static const char alpha[] = "abcxABZ09_ -./\t\n\r]}";
  int n = rnd(maxlen + 1);
  std::string s;
  for (int i = 0; i < n; ++i) {
    if (rnd(16) == 0) s.push_back((char)rnd(256));
    else s.push_back(alpha[rnd(sizeof(alpha) - 1)]);
  }
  return s;
}

static std::string noisy_pattern() {
  static const char alpha[] = "ab-^$.*+?{}[]()|\\:=,0129dwsDbBcxu";
  int n = 1 + rnd(10);
  std::string s;
  for (int i = 0; i < n; ++i) s.push_back(alpha[rnd(sizeof(alpha) - 1)]);
  return s;
}

struct Stats {
  long checked = 0, mism = 0, rejected = 0, unsup = 0;
};

static void report(Stats& st, const std::string& what, const std::string& p, const std::string& s, int a, int b) {
  if (++st.mism <= 10)
    fprintf(stderr, "MISMATCH %s pattern=%s input_len=%zu input=%s std=%d nfa=%d\n", what.c_str(), p.c_str(), s.size(),
            s.size() <= 64 ? s.c_str() : "(long)", a, b);
}

static void check_pattern(Stats& st, const std::string& p, const std::vector<std::string>& inputs, bool search) {
  std::regex r;
  bool std_ok = true;
  try {
    r = std::regex(p, std::regex::ECMAScript | std::regex::optimize);
  } catch (...) {
    std_ok = false;
  }
  nfa::Prog prog;
  int nfa_ok = 1;  // 1 ok, 0 syntax error, -1 unsupported
  try {
    prog = nfa::compile(p);
  } catch (const nfa::Unsupported&) {
    nfa_ok = -1;
  } catch (const nfa::SyntaxError&) {
    nfa_ok = 0;
  }
  if (nfa_ok < 0) {
    ++st.unsup;
    return;
  }
  ++st.checked;
  if (!std_ok || !nfa_ok) {
    if (std_ok != (nfa_ok == 1)) report(st, "accept", p, "", std_ok, nfa_ok);
    ++st.rejected;
    return;
  }
  nfa::Runner run;
  for (const auto& s : inputs) {
    ++st.checked;
    const auto* b = reinterpret_cast<const uint8_t*>(s.data());
    const int a = std::regex_match(s, r), m = run.run(prog, b, s.size(), false);
    if (a != m) report(st, "match", p, s, a, m);
    if (search) {
      const int a2 = std::regex_search(s, r), m2 = run.run(prog, b, s.size(), true);
      if (a2 != m2) report(st, "search", p, s, a2, m2);
    }
  }
}

// Nested-quantifier families (config 5's and classic blow-ups) on short
// subjects the backtracker still finishes.
static void nested(Stats& st, int n) {
  static const char* pats[] = {"(a|aa)*b", "(.{0,8}){1,8}foo", "((a*)*)*", "(a*b*)*c", "(?:a+)+b", "(x|y|xy)*z",
                               ".*(x|y).*(z|w).*q", "[a-z]*[a-z]*[a-z]*[a-z]*z", "(a?){3}a{3}", "((ab)*|a)*b?",
                               "(?:.{0,2}){2,3}o", "(\\w+\\.)*x"};
  for (int i = 0; i < n; ++i) {
    const std::string p = pats[rnd(sizeof(pats) / sizeof(*pats))];
    std::vector<std::string> in;
    for (int k = 0; k < 20; ++k) {
      std::string s;
      const int len = rnd(13);
      for (int j = 0; j < len; ++j) s.push_back("abxyzwqfo.\n"[rnd(12)]);
      in.push_back(s);
    }
    check_pattern(st, p, in, true);
  }
}

// Long subjects (1 - 8 KiB) on families whose backtracking cost stays
// polynomial of low degree for std::regex.
static void long_inputs(Stats& st, int n) {
  static const char* fams[] = {
      "x.*", ".*q", "[a-z]*z", "(ab|cd)*e", "a{0,8}b+", "(foo|bar)+", "[^/]*/.*", "/x1/.*q", "[a-z0-9._-]+",
      "(?:[a-c]{3})*d?", "\\w+\\.example", "(a|b|c|d)*", "[^#]*", "(?:/[a-z]+)+/?", "h(e|a)llo.*"};
  static const char alpha[] = "abcdefghijklmnopqrstuvwxyz0123456789-_./q#";
  for (int i = 0; i < n; ++i) {
    const std::string p = fams[rnd(sizeof(fams) / sizeof(*fams))];
    const int len = 1024 + rnd(8192 - 1024);
    std::string s;
    // mostly from a subject alphabet close to the pattern's, so both outcomes occur
    const int mode = rnd(4);
    for (int k = 0; k < len; ++k) {
      if (mode == 0) s.push_back(alpha[rnd(sizeof(alpha) - 1)]);
      else if (mode == 1) s.push_back("abcd"[rnd(4)]);
      else if (mode == 2) s.push_back("foobar"[rnd(6)]);
      else s.push_back("abcdefghijklmnopqrstuvwxyz"[rnd(26)]);
    }
    if (rnd(2)) s.back() = "qzebd"[rnd(5)];
    if (rnd(4) == 0) s = "/x1/" + s;
    check_pattern(st, p, {s}, false);
  }
}

int main(int argc, char** argv) {
  rng.seed(argc > 1 ? strtoull(argv[1], 0, 10) : 1);
  const int npat = argc > 2 ? atoi(argv[2]) : 2000;
  const int nstr = argc > 3 ? atoi(argv[3]) : 100;
  const int nlong = argc > 4 ? atoi(argv[4]) : 200;
  Stats st;
  for (int i = 0; i < npat; ++i) {
    bool qq = false;
    const std::string p = gen(0, &qq);
    std::vector<std::string> in;
    for (int k = 0; k < nstr; ++k) in.push_back(rand_input(10));
    check_pattern(st, p, in, true);
  }
  for (int i = 0; i < npat; ++i) check_pattern(st, noisy_pattern(), {"", "a", "ab", "-", "b0"}, true);
  nested(st, 200);
  long_inputs(st, nlong);
  printf("checked %ld mismatches %ld rejected %ld unsupported %ld\n", st.checked, st.mism, st.rejected, st.unsup);
  return st.mism ? 1 : 0;
}
