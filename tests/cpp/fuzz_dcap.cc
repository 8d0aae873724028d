// Differential fuzzer of the forced-capture analysis (regex_ecma.h
// analyze_dcap / DcapForm, program.h DcapSpec): for random patterns of the
// form [^] P1 (C{n,m}) L2 \1 R and near misses, whenever the analysis accepts
// a pattern, the first-pass decision -- P1, the maximal C-run with length in
// [n, m], L2, the run repeated, R's automaton over the rest -- must equal
// libstdc++ std::regex_match (the reference engine, envoy/cilium_network_policy.h:
// 68-71) on every subject.  Test infrastructure only.
//   fuzz_dcap <seed> <n_patterns> <subjects_per_pattern>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <regex>
#include <string>
#include <vector>

#include "../../cilium_amd/csrc/regex_ecma.h"

using namespace l7m::re;
static std::mt19937_64 rng;
static int rnd(int n) { return (int)(rng() % (uint64_t)n); }
template <class T, size_t N>
static const T& pick(const T (&a)[N]) { return a[rnd((int)N)]; }

static const char* kP1[] = {"", "/", "/api/", "x", "^/", "^", "ab", "\\/", "[/]"};
static const char* kG[] = {"(\\w+)", "([a-c]*)", "(\\d{2,3})", "([^/]+)", "(.)", "([a-z]{1,4})", "(\\w)",
                           "([ab]?)", "(\\d{0,})", "(x+?)", "([^-]*)", "(a|b)", "((a)+)", "(\\w+)+"};
static const char* kL2[] = {"/", "-", "--", "/x", ".", "\\.", "", "a", "[/]", "/?"};
static const char* kR[] = {"", "(/.*)?", "\\.json", "[0-9]*$", "/[a-z]+", "(x|yz)*", "$", "\\b", "(?=x)x",
                           "\\1", ".*", "(/\\w+)*"};

static std::string subject(const std::string& p1, bool good) {
  static const char* runs[] = {"a", "ab", "abc", "users", "12", "123", "1234", "x_1", "", "Zz9", "a.b", "b",
                               "-", "aa"};
  static const char* seps[] = {"/", "-", "--", "/x", ".", "", "a"};
  static const char* tails[] = {"", "/", "/x/y", ".json", "123", "xyz", "x", "/abc", "-", "yz"};
  std::string r1 = pick(runs), r2 = good ? r1 : pick(runs);
  if (rnd(6) == 0) r2 = r1 + "a";
  std::string s = (rnd(8) ? p1 : std::string(pick(kP1))) + r1 + pick(seps) + r2 + pick(tails);
  std::string out;
  for (char c : s) if (c != '^' && c != '\\' && c != '[' && c != ']' && c != '?') out.push_back(c);
  if (rnd(10) == 0) out = out.substr(0, rnd((int)out.size() + 1));
  return out;
}

static bool dfa_full(const Dfa& d, const std::string& s) {
  uint32_t st = d.start;
  for (unsigned char c : s) st = d.next[st * d.ncls + d.cmap[c]];
  for (uint32_t p : d.sets[d.endset[st]]) if (p == 0) return true;
  return false;
}

// The kernel's dcap_holds (l7m_http_impl.h) on the host.
static bool dcap_holds(const DcapForm& f, const Dfa* rd, const std::string& v) {
  const size_t l1 = f.p1.size(), l2 = f.l2.size();
  if (v.size() < l1 + l2 || v.compare(0, l1, f.p1) != 0) return false;
  size_t e = l1;
  while (e < v.size() && f.cls.test(static_cast<unsigned char>(v[e]))) ++e;
  const size_t r = e - l1;
  if (r < static_cast<size_t>(f.min) || (f.max >= 0 && r > static_cast<size_t>(f.max))) return false;
  if (e + l2 + r > v.size()) return false;
  if (v.compare(e, l2, f.l2) != 0 || v.compare(e + l2, r, v, l1, r) != 0) return false;
  const size_t t = e + l2 + r;
  if (!rd) return t == v.size();
  return dfa_full(*rd, v.substr(t));
}

int main(int argc, char** argv) {
  rng.seed(argc > 1 ? strtoull(argv[1], 0, 10) : 1);
  const int npat = argc > 2 ? atoi(argv[2]) : 2000;
  const int nstr = argc > 3 ? atoi(argv[3]) : 200;
  long accepted = 0, declined = 0, checked = 0, matched = 0, mism = 0;
  for (int i = 0; i < npat; ++i) {
    const std::string p1 = pick(kP1);
    std::string pat = p1 + pick(kG) + pick(kL2) + "\\1" + pick(kR);
    std::regex re;
    try { re = std::regex(pat, std::regex::ECMAScript); } catch (...) { continue; }
    Ast full;
    std::string err;
    if (parse_ecma(pat, &full, &err) != Status::Ok) continue;
    DcapForm f;
    if (!analyze_dcap(full, &f)) { ++declined; continue; }
    ++accepted;
    Dfa rd;
    if (!f.r_empty) {
      DfaLimits lim;
      if (build_dfa({&f.r}, lim, &rd) != Status::Ok) { printf("R-DFA %s\n", pat.c_str()); ++mism; continue; }
    }
    for (int j = 0; j < nstr; ++j) {
      const std::string s = subject(p1, rnd(2) == 0);
      const bool ref = std::regex_match(s, re);
      const bool got = dcap_holds(f, f.r_empty ? nullptr : &rd, s);
      ++checked;
      matched += ref;
      if (ref != got) {
        ++mism;
        if (mism < 20) printf("MISMATCH pat=%s in=%s ref=%d got=%d\n", pat.c_str(), s.c_str(), ref, got);
      }
    }
  }
  printf("accepted=%ld declined=%ld checked=%ld matched=%ld mismatches=%ld\n", accepted, declined, checked, matched,
         mism);
  return mism || !accepted || !matched ? 1 : 0;
}
