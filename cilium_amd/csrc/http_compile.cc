// http_compile.cc — compile []PortRuleHTTP into the HTTP device program.
//
// Pipeline (cold path, once per policy revision):
//   1. getHTTPRule (pkg/envoy/server.go:261-320): PortRuleHTTP -> HeaderMatcher
//      list, sorted by SortHeaderMatchers (pkg/envoy/sort.go:205-250).  Equal
//      (Name, Value) pairs involving a header matcher make Go dereference a nil
//      Regex and panic (sort.go:225-228); we return L7M_EINVAL_RULE instead.
//   2. Envoy HeaderData (envoy/cilium_network_policy.h:52-66 -> upstream
//      ConfigUtility::HeaderData): name lower-cased; empty value -> Present,
//      regex flag -> Regex (std::regex(value, optimize): throws -> NACK, here
//      L7M_EINVAL_REGEX), else exact Value.
//   3. Fields: ":method", ":path", ":authority", then every other header name
//      a rule references.  Per field, the distinct Regex/Value patterns are
//      determinised together into DFA groups (split when a group exceeds the
//      state/table limits); a header-name DFA maps request header names to
//      field ids.
//   4. First-match index: every rule is "keyed" on its most selective matcher.
//      For each (DFA, end set) the sorted list of rules keyed on a pattern of
//      that set is precomputed; at run time the kernel scans those lists in
//      rule order and verifies the rule's remaining matchers (AND), giving the
//      smallest matching rule index = HttpNetworkPolicyRule OR semantics
//      (envoy/cilium_network_policy.h:98-105) with a deterministic index.
#include <algorithm>
#include <cstring>
#include <map>
#include <regex>
#include <unordered_map>

#include "dfa_pack.h"
#include "l7m_internal.h"
#include "program.h"
#include "regex_ecma.h"
#include "regex_vm.h"

namespace l7m {
namespace {

std::string cstr(const char* p) { return p ? std::string(p) : std::string(); }

// States of one look-ahead pattern's exact automaton before it is carried as
// a superset (the look-ahead dropped) and decided by the slow path.
constexpr size_t kLookMaxStates = 1u << 16;

// Go strings.SplitN(s, " ", 2)
std::vector<std::string> split2(const std::string& s) {
  size_t k = s.find(' ');
  if (k == std::string::npos) return {s};
  return {s.substr(0, k), s.substr(k + 1)};
}

// Go strings.TrimRight(s, ":")
std::string trim_right_colon(std::string s) {
  while (!s.empty() && s.back() == ':') s.pop_back();
  return s;
}

// HeaderMatcherLess (pkg/envoy/sort.go:209-233) without the nil dereference;
// the caller rejects the inputs where Go would panic.
bool matcher_less(const HeaderMatcher& a, const HeaderMatcher& b) {
  if (a.name != b.name) return a.name < b.name;
  if (a.value != b.value) return a.value < b.value;
  bool ar = a.has_regex && a.regex, br = b.has_regex && b.regex;
  return !ar && br;
}

struct FieldPattern {
  MatchKind kind;
  std::string value;
  bool operator<(const FieldPattern& o) const {
    if (kind != o.kind) return kind < o.kind;
    return value < o.value;
  }
};

// Search automaton of <= kSearchMaxPats RE2-dialect patterns (program.h
// kDfaSearch): the dense DFA of [\x00-\xff]*(p0|...|pk) with, per state, the
// patterns matching a substring that ends there (mid set, '$' unsatisfied)
// and at the end of the input (end set).
struct SearchDfa {
  uint32_t nstates = 0, ncls = 0, start = 0, start_mid = 0;
  uint8_t cmap[256] = {0};
  std::vector<uint32_t> table;    // nstates * ncls: next state | mid id << 24
  std::vector<uint32_t> endmask;  // per state
  std::vector<uint32_t> midmask;  // per mid id (0: no pattern)
};

re::Status build_search_dfa(const std::vector<const re::Ast*>& pats, SearchDfa* out) {
  if (pats.size() > kSearchMaxPats) return re::Status::TooBig;
  std::vector<re::Ast> a(pats.size());
  std::vector<const re::Ast*> ptrs;
  for (size_t i = 0; i < pats.size(); ++i) {
    a[i] = *pats[i];
    re::simplify_search(&a[i]);
    re::make_search_prefix(&a[i]);
    ptrs.push_back(&a[i]);
  }
  re::Dfa d;
  re::DfaLimits lim;
  lim.max_states = 1u << 17;
  lim.max_table_bytes = 32ull << 20;
  const re::Status st = re::build_dfa(ptrs, lim, &d, /*with_mid=*/true);
  if (st != re::Status::Ok) return st;
  if (static_cast<uint64_t>(d.nstates) * d.ncls >= (1u << 24)) return re::Status::TooBig;
  std::vector<uint32_t> set_mask(d.sets.size(), 0);
  for (size_t k = 0; k < d.sets.size(); ++k)
    for (uint32_t p : d.sets[k]) set_mask[k] |= 1u << p;
  // mid ids: distinct mid sets, 0 = the empty set
  std::vector<uint32_t> mid_id(d.sets.size(), kNone);
  out->midmask.assign(1, 0u);
  mid_id[0] = 0;
  for (int q = 0; q < d.nstates; ++q) {
    const uint32_t sid = d.midset[q];
    if (mid_id[sid] != kNone) continue;
    if (out->midmask.size() >= kSearchMaxMid) return re::Status::TooBig;
    mid_id[sid] = static_cast<uint32_t>(out->midmask.size());
    out->midmask.push_back(set_mask[sid]);
  }
  out->nstates = static_cast<uint32_t>(d.nstates);
  out->ncls = static_cast<uint32_t>(d.ncls);
  out->start = static_cast<uint32_t>(d.start);
  out->start_mid = set_mask[d.midset[d.start]];
  std::memcpy(out->cmap, d.cmap, 256);
  out->table.resize(static_cast<size_t>(d.nstates) * d.ncls);
  for (size_t i = 0; i < out->table.size(); ++i) {
    const uint32_t nx = d.next[i];
    out->table[i] = nx | mid_id[d.midset[nx]] << 24;
  }
  out->endmask.resize(d.nstates);
  for (int q = 0; q < d.nstates; ++q) out->endmask[q] = set_mask[d.endset[q]];
  return re::Status::Ok;
}

struct Group {
  std::vector<uint32_t> pats;  // field pattern indices (local id = position)
  PackedDfa pk;                // kDfaPacked groups
  bool search = false;         // kDfaSearch group (sd)
  SearchDfa sd;
  bool alit = false;           // kDfaAlit group (no automaton: the field's alit scan)
};

// Literal-anchored RE2 patterns of one field (program.h FieldDesc::alit_*).
struct AlitField {
  bool on = false;
  uint32_t first_group = 0;            // field group index of the first kDfaAlit group
  std::vector<uint32_t> tab;           // buckets x {gram, pattern + 1, gram, pattern + 1}
  std::vector<uint32_t> pats;          // field pattern ids in alit order (AlitRec order)
  std::vector<std::string> lit;        // per alit pattern: L
  std::vector<uint32_t> k;             // per alit pattern: offset of its table gram in L
  std::vector<uint32_t> resid;         // per alit pattern: residual id, kNone = empty
  PackedDfa resid_pk;                  // automaton of the distinct residuals
  uint32_t n_resid = 0;
};

// Choose the alit patterns of a field: every RE2 pattern L R whose L's
// grams fit the table (rarest gram first); the rest stay search patterns.
void plan_alit(const std::vector<re::Ast>& asts, const std::vector<uint32_t>& sidx, AlitField* out,
               std::vector<uint32_t>* rest) {
  std::vector<uint32_t> cand;
  std::vector<std::string> lits;
  std::vector<re::Ast> res;
  for (uint32_t p : sidx) {
    re::Ast sa = asts[p];
    re::simplify_search(&sa);
    std::string L;
    re::Ast R;
    if (re::split_literal_prefix(sa, &L, &R)) {
      cand.push_back(p);
      lits.push_back(std::move(L));
      res.push_back(std::move(R));
    } else {
      rest->push_back(p);
    }
  }
  if (cand.size() < kAlitMinPatterns) {
    rest->insert(rest->end(), cand.begin(), cand.end());
    std::sort(rest->begin(), rest->end());
    return;
  }
  std::map<uint32_t, uint32_t> freq;
  for (const auto& L : lits)
    for (size_t i = 0; i + 4 <= L.size(); ++i) {
      uint32_t g;
      std::memcpy(&g, L.data() + i, 4);
      ++freq[g];
    }
  uint32_t buckets = 64;
  while (buckets < 2 * cand.size()) buckets <<= 1;  // quarter-full: every pattern finds a bucket
  if (16ull * buckets > kAlitMaxLdsBytes) buckets = kAlitMaxLdsBytes / 16;
  out->tab.assign(4ull * buckets, 0u);
  std::map<std::string, uint32_t> rid;
  std::vector<re::Ast> rasts;
  for (size_t c = 0; c < cand.size(); ++c) {
    const std::string& L = lits[c];
    int best_i = -1, best_e = -1;
    uint32_t best_f = kNone, best_g = 0;
    for (size_t i = 0; i + 4 <= L.size(); ++i) {
      uint32_t g;
      std::memcpy(&g, L.data() + i, 4);
      const uint32_t* b = &out->tab[4ull * (gram_bucket(g) & (buckets - 1))];
      const int e = !b[1] ? 0 : !b[3] ? 1 : -1;
      if (e < 0) continue;
      if (freq[g] < best_f) {
        best_f = freq[g];
        best_i = static_cast<int>(i);
        best_e = e;
        best_g = g;
      }
    }
    if (best_i < 0) {  // every bucket of its grams is full: a search pattern
      rest->push_back(cand[c]);
      continue;
    }
    const uint32_t id = static_cast<uint32_t>(out->pats.size());
    uint32_t* b = &out->tab[4ull * (gram_bucket(best_g) & (buckets - 1))];
    b[2 * best_e] = best_g;
    b[2 * best_e + 1] = id + 1;
    out->pats.push_back(cand[c]);
    out->lit.push_back(L);
    out->k.push_back(static_cast<uint32_t>(best_i));
    if (re::residual_is_empty(res[c])) {
      out->resid.push_back(kNone);
    } else {
      auto it = rid.emplace(re::ast_key(res[c]), static_cast<uint32_t>(rasts.size()));
      if (it.second) rasts.push_back(std::move(res[c]));
      out->resid.push_back(it.first->second);
    }
  }
  std::sort(rest->begin(), rest->end());
  if (out->pats.size() < kAlitMinPatterns) {
    rest->insert(rest->end(), out->pats.begin(), out->pats.end());
    std::sort(rest->begin(), rest->end());
    *out = AlitField();
    return;
  }
  out->n_resid = static_cast<uint32_t>(rasts.size());
  if (!rasts.empty()) {
    std::vector<const re::Ast*> rp;
    for (const auto& a : rasts) rp.push_back(&a);
    if (build_field_dfa(rp, FieldDfaLimits(), &out->resid_pk) != re::Status::Ok || out->resid_pk.n_slots > 12000) {
      rest->insert(rest->end(), out->pats.begin(), out->pats.end());  // residual automaton too large: search groups
      std::sort(rest->begin(), rest->end());
      *out = AlitField();
      return;
    }
  }
  out->on = true;
}

// Search groups of one field's RE2-dialect patterns: chunks of
// kSearchMaxPats, halved while an automaton exceeds the limits.
int build_search_groups(const std::vector<const re::Ast*>& asts, std::vector<uint32_t> idx,
                        std::vector<Group>* out, std::string* err) {
  if (idx.size() > kSearchMaxPats) {
    for (size_t o = 0; o < idx.size(); o += kSearchMaxPats) {
      std::vector<uint32_t> part(idx.begin() + o, idx.begin() + std::min(idx.size(), o + kSearchMaxPats));
      const int rc = build_search_groups(asts, std::move(part), out, err);
      if (rc != L7M_OK) return rc;
    }
    return L7M_OK;
  }
  std::vector<const re::Ast*> sub;
  for (uint32_t i : idx) sub.push_back(asts[i]);
  Group g;
  g.search = true;
  const re::Status st = build_search_dfa(sub, &g.sd);
  if (st == re::Status::Ok) {
    g.pats = std::move(idx);
    out->push_back(std::move(g));
    return L7M_OK;
  }
  if (st != re::Status::TooBig) {
    *err = "search DFA construction failed";
    return L7M_EUNSUPPORTED;
  }
  if (idx.size() == 1) {
    *err = "a single search pattern exceeds the DFA state limit";
    return L7M_ETOOBIG;
  }
  const size_t h = idx.size() / 2;
  std::vector<uint32_t> a(idx.begin(), idx.begin() + h), b(idx.begin() + h, idx.end());
  const int rc = build_search_groups(asts, std::move(a), out, err);
  if (rc != L7M_OK) return rc;
  return build_search_groups(asts, std::move(b), out, err);
}

// RE2-dialect gram filter of one field (program.h FieldDesc::gram_tab): a
// 2-entry-bucket table 4-byte gram -> mask of search groups (bit j % 32 of
// the field's search group j).  Each pattern with a required literal is
// entered under ONE of its literal's grams -- the rarest among the field's
// patterns whose bucket has room --, so a value that contains none of a
// group's chosen grams cannot match any of the group's patterns and the
// group's automaton is not walked.
struct GramFilter {
  bool on = false;
  uint32_t search_first = 0;  // field group index of the first search group
  uint32_t always = 0;        // groups walked for every value
  uint32_t n_search = 0;      // search groups of the field
  std::vector<uint32_t> tab;  // buckets x {gram, mask, gram, mask}
};

void build_gram_filter(const std::vector<Group>& groups, uint32_t first, uint32_t first_lit,
                       const std::vector<std::vector<uint32_t>>& grams, GramFilter* out) {
  const uint32_t ns = static_cast<uint32_t>(groups.size()) - first;
  out->search_first = first;
  if (ns < kGramMinGroups || ns > kGramMaxGroups || first_lit == groups.size()) return;
  std::map<uint32_t, uint32_t> freq;
  uint32_t n_lit = 0;
  for (uint32_t j = first_lit; j < groups.size(); ++j)
    for (uint32_t p : groups[j].pats) {
      for (uint32_t g : grams[p]) ++freq[g];
      ++n_lit;
    }
  uint32_t buckets = 64;
  while (buckets < n_lit) buckets <<= 1;
  if (buckets > 65536) return;
  out->tab.assign(4ull * buckets, 0u);
  for (uint32_t j = first; j < first_lit; ++j) out->always |= 1u << ((j - first) & 31u);
  for (uint32_t j = first_lit; j < groups.size(); ++j) {
    const uint32_t bit = 1u << ((j - first) & 31u);
    for (uint32_t p : groups[j].pats) {
      uint32_t best = kNone, best_freq = kNone;
      int best_slot = -1;
      for (uint32_t g : grams[p]) {
        uint32_t* b = &out->tab[4ull * (gram_bucket(g) & (buckets - 1))];
        int slot = -1;
        for (int e = 0; e < 2 && slot < 0; ++e)
          if (b[2 * e + 1] && b[2 * e] == g) slot = e;  // already entered: shares the entry
        for (int e = 0; e < 2 && slot < 0; ++e)
          if (!b[2 * e + 1]) slot = e;
        if (slot < 0) continue;
        const uint32_t fq = freq[g];
        if (fq < best_freq) {
          best = g;
          best_freq = fq;
          best_slot = slot;
        }
      }
      if (best_slot < 0) {  // every bucket of its grams is full: walk the group always
        out->always |= bit;
        continue;
      }
      uint32_t* b = &out->tab[4ull * (gram_bucket(best) & (buckets - 1))];
      b[2 * best_slot] = best;
      b[2 * best_slot + 1] |= bit;
    }
  }
  out->on = true;
}

// Build the field automata of one field's patterns: normally ONE automaton
// (dfa_pack.h, linear in the rules for prefix-diverging sets); a set whose
// product exceeds the limits (e.g. unanchored RE2-search patterns, which never
// latch) is split in halves.
int build_groups(const std::vector<const re::Ast*>& asts, std::vector<uint32_t> idx,
                 const FieldDfaLimits& lim, std::vector<Group>* out, std::string* err) {
  std::vector<const re::Ast*> sub;
  for (uint32_t i : idx) sub.push_back(asts[i]);
  Group g;
  re::Status st = build_field_dfa(sub, lim, &g.pk);
  if (st == re::Status::Ok) {
    g.pats = std::move(idx);
    out->push_back(std::move(g));
    return L7M_OK;
  }
  if (st != re::Status::TooBig) {
    *err = "DFA construction failed";
    return L7M_EUNSUPPORTED;
  }
  if (idx.size() == 1) {
    *err = "a single pattern exceeds the DFA state/table limit";
    return L7M_ETOOBIG;
  }
  size_t h = idx.size() / 2;
  std::vector<uint32_t> a(idx.begin(), idx.begin() + h), b(idx.begin() + h, idx.end());
  int rc = build_groups(asts, std::move(a), lim, out, err);
  if (rc != L7M_OK) return rc;
  return build_groups(asts, std::move(b), lim, out, err);
}

}  // namespace

std::string lower_ascii(const std::string& s) {
  std::string r = s;
  for (auto& c : r)
    if (c >= 'A' && c <= 'Z') c = static_cast<char>(c - 'A' + 'a');
  return r;
}

MatchKind envoy_kind(const HeaderMatcher& m) {
  if (m.value.empty()) return MatchKind::Present;
  if (m.has_regex && m.regex) return MatchKind::Regex;
  return MatchKind::Value;
}

int translate_http_rule(const l7m_http_rule& r, std::vector<HeaderMatcher>* out, std::string* err) {
  out->clear();
  std::string path = cstr(r.path), method = cstr(r.method), host = cstr(r.host);
  if (!path.empty()) out->push_back({":path", path, true, true});
  if (!method.empty()) out->push_back({":method", method, true, true});
  if (!host.empty()) out->push_back({":authority", host, true, true});
  for (uint32_t j = 0; j < r.n_headers; ++j) {
    if (!r.headers) {
      *err = "headers == NULL with n_headers > 0";
      return L7M_EINVAL;
    }
    auto parts = split2(cstr(r.headers[j]));
    if (parts.size() == 2) out->push_back({trim_right_colon(parts[0]), parts[1], false, false});
    else out->push_back({parts[0], "", false, false});
  }
  // SortHeaderMatchers panics on equal (Name, Value) with a nil Regex.
  for (size_t a = 0; a < out->size(); ++a)
    for (size_t b = a + 1; b < out->size(); ++b) {
      const auto& x = (*out)[a];
      const auto& y = (*out)[b];
      if (x.name == y.name && x.value == y.value && !(x.has_regex && y.has_regex)) {
        *err = "duplicate header matcher '" + x.name + "' (getHTTPRule sort would panic, "
               "pkg/envoy/sort.go:225-228)";
        return L7M_EINVAL_RULE;
      }
    }
  std::stable_sort(out->begin(), out->end(), matcher_less);
  for (const auto& m : *out)
    if (m.name.empty()) {
      // Envoy's HeaderMatcher.name validation (min_bytes 1) rejects the policy.
      *err = "empty header name";
      return L7M_EINVAL_RULE;
    }
  return L7M_OK;
}

namespace {

constexpr size_t kLitMinBytes = 16;  // shorter literal values are walked byte by byte

// no_alit: fields whose literal-anchored scan is turned off (their patterns
// stay search groups); set by compile_http_plan when a field's bucket table
// does not fit the LDS budget.  *alit_over receives such a field.
CompileResult compile_http_core(const l7m_http_rule* rules, size_t n, const PolicyPlan& plan, const l7m_opts& opts,
                                uint64_t no_alit, uint32_t* alit_over) {
  CompileResult res;
  auto fail = [&](int st, const std::string& m) {
    res.status = st;
    res.err = m;
    return res;
  };
  if (n > 0 && !rules) return fail(L7M_EINVAL, "rules == NULL");
  const bool re2 = opts.dialect == L7M_DIALECT_RE2_SEARCH;
  if (opts.dialect != L7M_DIALECT_ENVOY_ECMA_FULL && !re2) return fail(L7M_EINVAL, "unknown dialect");
  if (n >= kNone / 2) return fail(L7M_ETOOBIG, "too many rules");

  // 1-2. translate, field/pattern assignment
  std::vector<std::string> field_names = {":method", ":path", ":authority"};
  std::unordered_map<std::string, uint32_t> field_of = {
      {":method", kFieldMethod}, {":path", kFieldPath}, {":authority", kFieldAuthority}};
  std::vector<std::map<FieldPattern, uint32_t>> fpat_idx(3);
  std::vector<std::vector<FieldPattern>> fpats(3);

  struct RM {
    uint32_t field;
    MatchKind kind;
    uint32_t fpat;  // field pattern index (kNone for Present)
  };
  std::vector<std::vector<RM>> rule_m(n);
  std::vector<HeaderMatcher> hm;
  for (size_t i = 0; i < n; ++i) {
    std::string err;
    int rc = translate_http_rule(rules[i], &hm, &err);
    if (rc != L7M_OK) return fail(rc, "rule " + std::to_string(i) + ": " + err);
    if (hm.size() > kCrMaxMatchers)
      return fail(L7M_ETOOBIG, "rule " + std::to_string(i) + ": more than 255 header matchers");
    for (const auto& m : hm) {
      std::string lname = lower_ascii(m.name);  // Envoy LowerCaseString
      auto it = field_of.find(lname);
      uint32_t f;
      if (it == field_of.end()) {
        f = static_cast<uint32_t>(field_names.size());
        if (f >= kMaxFields)
          return fail(L7M_ETOOBIG, "more than 64 distinct header fields referenced");
        field_of.emplace(lname, f);
        field_names.push_back(lname);
        fpat_idx.emplace_back();
        fpats.emplace_back();
      } else {
        f = it->second;
      }
      MatchKind k = envoy_kind(m);
      RM r{f, k, kNone};
      if (k != MatchKind::Present) {
        FieldPattern fp{k, m.value};
        auto pit = fpat_idx[f].find(fp);
        if (pit == fpat_idx[f].end()) {
          pit = fpat_idx[f].emplace(fp, static_cast<uint32_t>(fpats[f].size())).first;
          fpats[f].push_back(fp);
        }
        r.fpat = pit->second;
      }
      rule_m[i].push_back(r);
    }
  }
  const uint32_t nf = static_cast<uint32_t>(field_names.size());

  // 3. parse patterns and build DFA groups per field
  FieldDfaLimits lim;
  if (opts.max_dfa_states) lim.max_multi_states = opts.max_dfa_states;
  if (opts.max_table_bytes) lim.max_slots = std::min<uint64_t>(lim.max_slots, opts.max_table_bytes / 4);
  std::vector<std::vector<Group>> groups(nf);
  // slow-path programs (regex_vm.h) of the patterns whose automata are
  // supersets (back-references, oversized look-ahead): [field][pattern]
  std::vector<std::vector<std::vector<uint32_t>>> slow_vm(nf);
  // back-references whose capture is forced (regex_ecma.h DcapForm): decided
  // in the first pass; [field][pattern] -> dcap id, kNone otherwise
  std::vector<std::vector<uint32_t>> dcap_of(nf);
  struct DcapOut {
    uint32_t field;
    re::DcapForm form;
    PackedDfa rpk;  // R's full-match automaton (unless form.r_empty)
  };
  std::vector<DcapOut> dcaps;
  // field pattern -> (group, local id)
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> fp_loc(nf);
  std::vector<GramFilter> gram(nf);  // RE2 dialect: per field, which search groups a value may need
  std::vector<AlitField> alit(nf);   // RE2 dialect: per field, the literal-anchored patterns
  for (uint32_t f = 0; f < nf; ++f) {
    if (fpats[f].empty()) continue;
    std::vector<re::Ast> asts(fpats[f].size());
    std::vector<const re::Ast*> ptrs;
    slow_vm[f].resize(fpats[f].size());
    dcap_of[f].assign(fpats[f].size(), kNone);
    for (size_t p = 0; p < fpats[f].size(); ++p) {
      const auto& fp = fpats[f][p];
      if (fp.kind == MatchKind::Regex && re2) {
        // Go regexp.MustCompile(p).MatchString(v): RE2 syntax, unanchored.
        std::string perr;
        re::Status st = re::parse_re2(fp.value, &asts[p], &perr);
        if (st == re::Status::Syntax)
          return fail(L7M_EINVAL_REGEX, "invalid regex '" + fp.value + "' on " + field_names[f] + ": " + perr +
                                            " (regexp.Compile would fail)");
        if (st != re::Status::Ok)
          return fail(L7M_EUNSUPPORTED, "regex '" + fp.value + "': " + perr + " is outside the RE2 byte subset");
      } else if (fp.kind == MatchKind::Regex) {
        try {
          std::regex probe(fp.value, std::regex::ECMAScript | std::regex::optimize);
          (void)probe;
        } catch (const std::regex_error& e) {
          return fail(L7M_EINVAL_REGEX, "invalid regex '" + fp.value + "' on " + field_names[f] +
                                            ": " + e.what() + " (Envoy would NACK the policy)");
        }
        std::string perr;
        re::Ast full;
        re::Status st = re::parse_ecma(fp.value, &full, &perr);
        if (st == re::Status::TooBig)
          return fail(L7M_ETOOBIG, "regex '" + fp.value + "': " + perr);
        if (st != re::Status::Ok)
          return fail(L7M_EUNSUPPORTED, "regex '" + fp.value + "': " + perr + " (parser disagrees with std::regex)");
        bool exact = true;
        asts[p] = re::lower_for_dfa(full, &exact);
        if (exact && re::has_node(asts[p], re::Node::Look)) {
          // look-ahead is determinised exactly (regex_ecma.cc build_ctx)
          // unless its automaton exceeds kLookMaxStates: then the DFA carries
          // the pattern without it (a superset) and the slow path decides
          re::Dfa probe;
          re::DfaLimits ll;
          ll.max_states = kLookMaxStates;
          if (re::build_dfa({&asts[p]}, ll, &probe) != re::Status::Ok) {
            asts[p] = re::drop_lookahead(asts[p]);
            exact = false;
          }
        }
        re::DcapForm form;
        if (!exact && dcaps.size() < kMaxDcap && re::analyze_dcap(full, &form)) {
          // a forced capture: the superset automaton plus byte compares in
          // the first pass decide it exactly (no slow path)
          DcapOut dc;
          dc.field = f;
          dc.form = std::move(form);
          if (!dc.form.r_empty) {
            std::vector<const re::Ast*> rp{&dc.form.r};
            if (build_field_dfa(rp, FieldDfaLimits(), &dc.rpk) != re::Status::Ok) dc.field = kNone;
          }
          if (dc.field != kNone) {
            dcap_of[f][p] = static_cast<uint32_t>(dcaps.size());
            dcaps.push_back(std::move(dc));
            exact = true;
          }
        }
        if (!exact) {
          // the automaton accepts a superset; rules using this pattern are
          // decided by the slow path (libstdc++'s executor restated)
          std::string verr;
          if (!vm_compile(full, &slow_vm[f][p], &verr))
            return fail(L7M_ETOOBIG, "regex '" + fp.value + "': " + verr);
        }
      } else {
        asts[p] = re::literal_ast(fp.value);
      }
      ptrs.push_back(&asts[p]);
    }
    // RE2 dialect: regex patterns become search automata (program.h
    // kDfaSearch); literal header values stay full-match packed automata
    std::vector<uint32_t> idx, sidx;
    for (uint32_t p = 0; p < fpats[f].size(); ++p)
      (re2 && fpats[f][p].kind == MatchKind::Regex ? sidx : idx).push_back(p);
    std::string err;
    if (!idx.empty()) {
      int rc = build_groups(ptrs, idx, lim, &groups[f], &err);
      if (rc != L7M_OK) return fail(rc, field_names[f] + ": " + err);
    }
    if (!sidx.empty()) {
      // literal-anchored patterns (L R) leave the search groups: an alit scan
      // decides them (gram probe, literal compare, shared residual automaton)
      {
        std::vector<uint32_t> rest;
        if (f < 64 && (no_alit >> f & 1)) rest = sidx;
        else plan_alit(asts, sidx, &alit[f], &rest);
        sidx = std::move(rest);
      }
      // patterns without a 4-byte required literal ("always" walked) are
      // grouped apart from the others, so the gram filter can skip whole groups
      std::vector<std::vector<uint32_t>> grams(fpats[f].size());
      std::vector<uint32_t> s_always, s_lit;
      for (uint32_t p : sidx) {
        for (const std::string& lit : re::required_literals(asts[p]))
          for (size_t i = 0; i + 4 <= lit.size(); ++i) {
            uint32_t g;
            std::memcpy(&g, lit.data() + i, 4);
            grams[p].push_back(g);
          }
        std::sort(grams[p].begin(), grams[p].end());
        grams[p].erase(std::unique(grams[p].begin(), grams[p].end()), grams[p].end());
        (grams[p].empty() ? s_always : s_lit).push_back(p);
      }
      const uint32_t first = static_cast<uint32_t>(groups[f].size());
      gram[f].search_first = first;
      if (sidx.empty()) {
        // every regex of the field is literal-anchored
      } else if (sidx.size() <= kSearchMaxPats && !alit[f].on) {  // one group: walked anyway, no filter
        int rc = build_search_groups(ptrs, sidx, &groups[f], &err);
        if (rc != L7M_OK) return fail(rc, field_names[f] + ": " + err);
        gram[f].search_first = first;
      } else {
        if (!s_always.empty()) {
          int rc = build_search_groups(ptrs, s_always, &groups[f], &err);
          if (rc != L7M_OK) return fail(rc, field_names[f] + ": " + err);
        }
        const uint32_t first_lit = static_cast<uint32_t>(groups[f].size());
        if (!s_lit.empty()) {
          int rc = build_search_groups(ptrs, s_lit, &groups[f], &err);
          if (rc != L7M_OK) return fail(rc, field_names[f] + ": " + err);
        }
        build_gram_filter(groups[f], first, first_lit, grams, &gram[f]);
      }
      gram[f].n_search = static_cast<uint32_t>(groups[f].size()) - first;
    }
    if (alit[f].on) {  // kDfaAlit groups of <= kSearchMaxPats patterns, after the search groups
      alit[f].first_group = static_cast<uint32_t>(groups[f].size());
      for (size_t o = 0; o < alit[f].pats.size(); o += kSearchMaxPats) {
        Group g;
        g.alit = true;
        g.pats.assign(alit[f].pats.begin() + o, alit[f].pats.begin() + std::min(alit[f].pats.size(), o + kSearchMaxPats));
        groups[f].push_back(std::move(g));
      }
    }
    fp_loc[f].assign(fpats[f].size(), {0, 0});
    for (uint32_t g = 0; g < groups[f].size(); ++g)
      for (uint32_t l = 0; l < groups[f][g].pats.size(); ++l)
        fp_loc[f][groups[f][g].pats[l]] = {g, l};
  }

  // header-name DFA over every regular field name (exact, lower-case)
  bool has_name = nf > 3;
  PackedDfa name_dfa;
  if (has_name) {
    std::vector<re::Ast> asts;
    for (uint32_t f = 3; f < nf; ++f) asts.push_back(re::literal_ast(field_names[f]));
    std::vector<const re::Ast*> ptrs;
    for (auto& a : asts) ptrs.push_back(&a);
    if (build_field_dfa(ptrs, FieldDfaLimits(), &name_dfa) != re::Status::Ok)
      return fail(L7M_ETOOBIG, "header-name DFA too large");
  }

  // global DFA numbering: fields in order, groups in order
  std::vector<uint32_t> dfa_first(nf, 0);
  uint32_t ndfa = 0;
  for (uint32_t f = 0; f < nf; ++f) {
    dfa_first[f] = ndfa;
    ndfa += static_cast<uint32_t>(groups[f].size());
  }

  // 4. keys: most selective matcher per rule
  std::vector<std::vector<uint32_t>> share(nf);
  for (uint32_t f = 0; f < nf; ++f) share[f].assign(fpats[f].size(), 0);
  for (size_t i = 0; i < n; ++i) {
    std::vector<std::pair<uint32_t, uint32_t>> seen;
    for (const auto& m : rule_m[i])
      if (m.fpat != kNone) {
        auto key = std::make_pair(m.field, m.fpat);
        if (std::find(seen.begin(), seen.end(), key) == seen.end()) {
          seen.push_back(key);
          share[m.field][m.fpat]++;
        }
      }
  }
  auto field_rank = [](uint32_t f) -> uint32_t {
    if (f == kFieldPath) return 0;
    if (f == kFieldAuthority) return 1;
    if (f == kFieldMethod) return 3;
    return 2;
  };
  // keyed lists
  std::vector<std::vector<std::vector<uint32_t>>> keyed(ndfa);  // [dfa][local pattern]
  for (uint32_t f = 0; f < nf; ++f)
    for (uint32_t g = 0; g < groups[f].size(); ++g)
      keyed[dfa_first[f] + g].resize(groups[f][g].pats.size());
  std::vector<std::vector<uint32_t>> pres_keyed(nf);
  uint32_t always_rule = kNone;
  std::vector<uint32_t> zero_list;  // no matchers, remote-restricted
  std::vector<std::vector<uint32_t>> remotes(n);
  bool any_remotes = true;
  for (size_t i = 0; i < n; ++i) {
    if (rules[i].n_remote_ids) {
      if (!rules[i].remote_ids) return fail(L7M_EINVAL, "remote_ids == NULL with n_remote_ids > 0");
      remotes[i].assign(rules[i].remote_ids, rules[i].remote_ids + rules[i].n_remote_ids);
      std::sort(remotes[i].begin(), remotes[i].end());
      remotes[i].erase(std::unique(remotes[i].begin(), remotes[i].end()), remotes[i].end());
      any_remotes = false;
    }
  }
  for (size_t i = 0; i < n; ++i) {
    if (rule_m[i].empty()) {
      // matcher-less rules: the smallest unrestricted one decides outright in a
      // one-entry map; otherwise they are checked like any other candidate
      // (remote set, port entry)
      if (plan.single && remotes[i].empty()) {
        if (always_rule == kNone) always_rule = static_cast<uint32_t>(i);
      } else {
        zero_list.push_back(static_cast<uint32_t>(i));
      }
      continue;
    }
    const RM* best = nullptr;
    auto score = [&](const RM& m) {
      uint64_t pres = m.kind == MatchKind::Present ? 1 : 0;
      uint64_t sh = m.fpat == kNone ? 0xffffffffu : share[m.field][m.fpat];
      return (pres << 60) | (sh << 8) | field_rank(m.field);
    };
    for (const auto& m : rule_m[i])
      if (!best || score(m) < score(*best)) best = &m;
    if (best->kind == MatchKind::Present) {
      pres_keyed[best->field].push_back(static_cast<uint32_t>(i));
    } else {
      auto loc = fp_loc[best->field][best->fpat];
      keyed[dfa_first[best->field] + loc.first][loc.second].push_back(static_cast<uint32_t>(i));
    }
  }

  // rules with slow-path matchers: (field, program) pairs, in matcher order
  std::vector<uint8_t> slow_rule(n, 0);
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> slow_list(n);  // (field, pattern)
  uint32_t n_slow = 0;
  for (size_t i = 0; i < n; ++i) {
    for (const auto& m : rule_m[i])
      if (m.fpat != kNone && !slow_vm[m.field][m.fpat].empty()) slow_list[i].push_back({m.field, m.fpat});
    if (!slow_list[i].empty()) {
      slow_rule[i] = 1;
      ++n_slow;
    }
  }

  // ---- assemble the program -------------------------------------------
  std::vector<uint32_t> pool;  // set pattern lists, remote ids
  auto push_list = [&](const std::vector<uint32_t>& v) -> Span {
    Span s{static_cast<uint32_t>(pool.size()), static_cast<uint32_t>(v.size())};
    pool.insert(pool.end(), v.begin(), v.end());
    return s;
  };
  // check records (program.h): one per (list, rule)
  std::vector<uint32_t> cr;
  auto push_records = [&](const std::vector<uint32_t>& rids) -> Span {
    Span s{static_cast<uint32_t>(cr.size()), static_cast<uint32_t>(rids.size())};
    for (uint32_t rid : rids) {
      cr.push_back(rid);
      cr.push_back(static_cast<uint32_t>(rule_m[rid].size()) | plan.rule_entry[rid] << kCrEntryShift |
                   (remotes[rid].empty() ? 0u : kCrRemote) | (slow_rule[rid] ? kCrSlow : 0u));
      for (const auto& m : rule_m[rid]) {
        uint32_t dfa = 0, pat = 0;
        if (m.fpat != kNone) {
          auto loc = fp_loc[m.field][m.fpat];
          dfa = dfa_first[m.field] + loc.first;
          pat = loc.second;
        }
        const uint32_t kind = m.kind == MatchKind::Present ? 1u : 0u;
        cr.push_back(m.field | (kind << 8) | (dfa << 9));
        if (m.fpat != kNone && dcap_of[m.field][m.fpat] != kNone) pat |= (dcap_of[m.field][m.fpat] + 1) << kDcapShift;
        cr.push_back(pat);
      }
    }
    return s;
  };
  if (ndfa >= (1u << 23)) return fail(L7M_ETOOBIG, "too many DFA groups");

  struct DfaOut {
    const PackedDfa* d;
    uint32_t field;
    uint32_t npats;
    const Group* grp;  // nullptr for the name DFA
  };
  std::vector<DfaOut> all;
  for (uint32_t f = 0; f < nf; ++f)
    for (auto& g : groups[f]) all.push_back({&g.pk, f, static_cast<uint32_t>(g.pats.size()), &g});
  if (has_name) all.push_back({&name_dfa, kNone, nf - 3, nullptr});
  // the literal-anchored fields' residual automata (after the name DFA)
  std::vector<uint32_t> resid_dfa(nf, kNone);
  for (uint32_t f = 0; f < nf; ++f)
    if (alit[f].on && alit[f].n_resid) {
      resid_dfa[f] = static_cast<uint32_t>(all.size());
      all.push_back({&alit[f].resid_pk, f, alit[f].n_resid, nullptr});
    }
  // forced-capture patterns' R automata (after those)
  std::vector<uint32_t> dcap_rdfa(dcaps.size(), kNone);
  for (size_t k = 0; k < dcaps.size(); ++k)
    if (!dcaps[k].form.r_empty) {
      dcap_rdfa[k] = static_cast<uint32_t>(all.size());
      all.push_back({&dcaps[k].rpk, dcaps[k].field, 1, nullptr});
    }
  const uint32_t ndt = static_cast<uint32_t>(all.size());

  std::vector<DfaDesc> dd(ndt);
  std::vector<Span> sets;
  std::vector<std::vector<Span>> ct(ndt);              // per DFA: [nsets + npats]
  std::vector<std::vector<uint64_t>> masks(ndt);       // per DFA with npats <= 64
  uint64_t total_states = 0;
  for (uint32_t k = 0; k < ndt; ++k) {
    const PackedDfa& d = *all[k].d;
    std::memset(&dd[k], 0, sizeof(DfaDesc));
    dd[k].start_base = d.start_base;
    dd[k].region = d.region;
    dd[k].start_latch = d.start_latch;
    dd[k].n_slots = d.n_slots;
    dd[k].nsets = static_cast<uint32_t>(d.sets.size());
    dd[k].npats = all[k].npats;
    dd[k].set_base = static_cast<uint32_t>(sets.size());
    dd[k].field = all[k].field;
    dd[k].nstates = d.nstates;
    dd[k].lds_table = dd[k].lds_es = dd[k].lds_latch = dd[k].lds_ct = dd[k].lds_mask = kNone;
    dd[k].lds_ctmask = kNone;
    dd[k].lit_tab = kNone;
    dd[k].lds_skip = kNone;
    dd[k].skip_lim = 0;
    dd[k].kind = kDfaPacked;
    dd[k].lds_search = dd[k].lds_mid = kNone;
    if (all[k].grp && all[k].grp->alit) {  // no automaton: codes from the field's alit scan
      dd[k].kind = kDfaAlit;
      dd[k].start_base = 0;
      dd[k].region = 0;
      dd[k].n_slots = 0;
      dd[k].nstates = 0;
    }
    if (all[k].grp && all[k].grp->search) {
      const SearchDfa& sd = all[k].grp->sd;
      dd[k].kind = kDfaSearch;
      dd[k].start_base = sd.start;
      dd[k].start_es8 = sd.start_mid;
      dd[k].region = 0;
      dd[k].n_slots = sd.nstates * sd.ncls;
      dd[k].nstates = sd.nstates;
      dd[k].acc_ncls = sd.ncls;
    }
    total_states += dd[k].nstates;
    for (size_t s = 0; s < d.sets.size(); ++s) {
      sets.push_back(push_list(d.sets[s]));
      if (k < ndfa) {
        std::vector<uint32_t> c;
        for (uint32_t p : d.sets[s]) {
          const auto& kl = keyed[k][p];
          c.insert(c.end(), kl.begin(), kl.end());
        }
        std::sort(c.begin(), c.end());
        c.erase(std::unique(c.begin(), c.end()), c.end());
        ct[k].push_back(push_records(c));
      }
      if (all[k].npats <= 64) {
        uint64_t m = 0;
        for (uint32_t p : d.sets[s]) m |= 1ull << p;
        masks[k].push_back(m);
      }
    }
    if (k < ndfa)
      for (uint32_t p = 0; p < all[k].npats; ++p) ct[k].push_back(push_records(keyed[k][p]));
  }
  std::vector<uint32_t> name_field;
  if (has_name) {
    for (const auto& s : name_dfa.sets) name_field.push_back(s.empty() ? kNone : 3 + s[0]);
  }
  std::vector<FieldDesc> fd(nf);
  for (uint32_t f = 0; f < nf; ++f) {
    fd[f].dfa_first = dfa_first[f];
    fd[f].ndfa = static_cast<uint32_t>(groups[f].size());
    fd[f].presence = push_records(pres_keyed[f]);
    fd[f].gram_tab = kNone;  // placed in the LDS image below
    fd[f].gram_mask = 0;
    fd[f].always = ~0u;
    fd[f].search_first = gram[f].search_first;
    fd[f].n_search = gram[f].n_search;
    fd[f].alit_tab = fd[f].alit_pats = kNone;
    fd[f].alit_mask = 0;
    fd[f].alit_lds = 0;
    fd[f].alit_granules = 0;
    fd[f].dcap_mask = 0;
    for (size_t k = 0; k < dcaps.size(); ++k)
      if (dcaps[k].field == f) fd[f].dcap_mask |= 1u << k;
    fd[f].resid_dfa = resid_dfa[f];
  }
  std::vector<Span> rremote(n);
  for (size_t i = 0; i < n; ++i) rremote[i] = push_list(remotes[i]);
  const Span zero_span = push_records(zero_list);
  cr.insert(cr.end(), 8, 0u);  // the kernel fetches 8 words per record

  // ---- LDS image: descriptors always; then, hottest DFA first (header
  // names, path, authority, method, header values), slot table + u16 end
  // codes/latches; then candidate tables and set masks, within the budget.
  // The kernel's LDS also holds the per-lane end-code columns (more than
  // kHttpRegDfas value DFAs: 4 bytes x kHttpBlock lanes each), the hit
  // counters (when they fit kMaxLdsCounters) and a record stage of at least
  // kHttpMinStage bytes per wave (l7m_kernels.hip http_lds_bytes).  What is
  // left bounds the table image; rule sets whose fixed part does not fit are
  // rejected here, when the policy loads, not on every batch.
  bool any_search = false;
  for (uint32_t f = 0; f < nf; ++f)
    for (const auto& g : groups[f]) any_search |= g.search;
  // (search programs keep their end codes in a global scratch, l7m_kernels.hip)
  const uint64_t codes_bytes = ndfa > kHttpRegDfas && !any_search ? 4ull * kHttpBlock * ndfa : 0;
  const uint64_t ctr_bytes = !kSliceHits && n + 2 <= kMaxLdsCounters ? 4ull * ((n + 2 + 3) & ~uint64_t(3)) : 0;
  const uint64_t stage_bytes = static_cast<uint64_t>(kHttpWaves) * (kHttpMinStage + 16);
  uint64_t img = 0;  // image words
  auto img_take = [&](uint64_t words) {
    uint64_t o = img;
    img += (words + 3) & ~uint64_t(3);  // 16-byte granules
    return static_cast<uint32_t>(o);
  };
  img_take(256);  // image words [0, 256): the zero dead row of every LDS slot table (program.h kLdsRowShift)
  const uint32_t lds_dfas = img_take(static_cast<uint64_t>(ndt) * sizeof(DfaDesc) / 4);
  const uint32_t lds_fields = img_take(static_cast<uint64_t>(nf) * sizeof(FieldDesc) / 4);
  const uint32_t lds_name_field = img_take(name_field.size());
  // forced-capture specs and their literals (read by every walk of their field)
  uint32_t lds_dcap = kNone;
  std::vector<uint32_t> dcap_p1(dcaps.size()), dcap_l2(dcaps.size());
  if (!dcaps.empty()) {
    lds_dcap = img_take(16ull * dcaps.size());
    for (size_t k = 0; k < dcaps.size(); ++k) {
      dcap_p1[k] = img_take((dcaps[k].form.p1.size() + 3) / 4);
      dcap_l2[k] = img_take((dcaps[k].form.l2.size() + 3) / 4);
    }
  }
  {
    const uint64_t fixed = 4 * img + codes_bytes + ctr_bytes + stage_bytes;
    if (fixed > kHttpLdsBytes)
      return fail(L7M_ETOOBIG, std::to_string(ndfa) + " value DFA groups over " + std::to_string(nf) +
                                   " fields need " + std::to_string(fixed) + " bytes of fixed LDS (descriptors, "
                                   "end-code columns, counters, record stage) > " + std::to_string(kHttpLdsBytes));
  }
  uint64_t budget_bytes = opts.lds_budget_bytes ? opts.lds_budget_bytes : kDefaultLdsBudget;
  {
    const uint64_t fixed = codes_bytes + ctr_bytes + stage_bytes;
    budget_bytes = std::min<uint64_t>(budget_bytes, fixed < kHttpLdsBytes ? kHttpLdsBytes - fixed : 0);
  }
  const uint64_t budget = budget_bytes / 4;
  // header-name table (always resident when it fits)
  uint32_t lds_name_tab = kNone, name_slots = 0;
  std::vector<uint32_t> name_off;
  if (has_name) {
    name_slots = 2;
    while (name_slots < 2 * (nf - 3)) name_slots <<= 1;
    uint64_t words = 4ull * name_slots;
    for (uint32_t f = 3; f < nf; ++f) words += ((field_names[f].size() + 3) / 4 + 3) & ~size_t(3);
    if (4 * words <= kMaxNameTabBytes && img + words <= budget) {
      lds_name_tab = img_take(4ull * name_slots);
      for (uint32_t f = 3; f < nf; ++f) name_off.push_back(img_take((field_names[f].size() + 3) / 4));
    }
  }
  // RE2-dialect literal-anchored patterns: the bucket table (read once per
  // value byte; their groups have no automaton, so it must be resident)
  for (uint32_t f = 0; f < nf; ++f) {
    if (!alit[f].on) continue;
    if (img + kAlitBloomWords + alit[f].tab.size() > budget) {
      // not resident: the caller compiles again with this field's patterns
      // as plain search groups (a policy that compiled before the alit scan
      // existed still compiles)
      *alit_over = f;
      return fail(L7M_ETOOBIG, field_names[f] + ": the literal-anchored pattern table needs " +
                                   std::to_string(4 * alit[f].tab.size()) + " bytes of LDS");
    }
    fd[f].alit_tab = img_take(kAlitBloomWords + alit[f].tab.size()) + kAlitBloomWords;  // prefilter bits, then the table
    fd[f].alit_mask = static_cast<uint32_t>(alit[f].tab.size() / 4 - 1);
  }
  // RE2-dialect gram filters (read once per value byte): right after the name table
  for (uint32_t f = 0; f < nf; ++f) {
    if (!gram[f].on || img + gram[f].tab.size() > budget) continue;
    fd[f].gram_tab = img_take(gram[f].tab.size());
    fd[f].gram_mask = static_cast<uint32_t>(gram[f].tab.size() / 4 - 1);
    fd[f].always = gram[f].always;
  }
  // search automata's mid masks (one read per value byte, <= 256 words each):
  // in LDS, so a search step costs one L2 request (the table entry), not two
  for (uint32_t k = 0; k < ndt; ++k) {
    if (!all[k].grp || !all[k].grp->search) continue;
    const uint64_t mw = all[k].grp->sd.midmask.size();
    if (img + ((mw + 3) & ~3ull) <= budget) dd[k].lds_mid = img_take(mw);
  }
  // ... the residual automata they walk (slot table + end codes, pattern masks)
  for (uint32_t f = 0; f < nf; ++f) {
    const uint32_t k = resid_dfa[f];
    if (k == kNone || fd[f].alit_tab == kNone) continue;
    const PackedDfa& d = *all[k].d;
    const uint64_t half_latch = (d.latch.size() + 1) / 2;
    const bool es8 = d.sets.size() < kEs8Latched && all[k].npats < kEs16Latched;
    if (es8 && img + d.n_slots <= kLdsTableWords &&
        img + ((d.n_slots + 3) & ~3ull) + ((half_latch + 3) & ~3ull) <= budget) {
      dd[k].lds_table = img_take(d.n_slots);
      dd[k].lds_es = kLdsEsInEntry;
      dd[k].lds_latch = 2 * img_take(half_latch);
    }
    if (!masks[k].empty() && img + ((2 * masks[k].size() + 3) & ~size_t(3)) <= budget)
      dd[k].lds_mask = img_take(2 * masks[k].size());
  }
  // (policy, direction, port) -> port entry table (open addressing on
  // ent_hash, program.h); in LDS when small
  uint32_t ent_slots = 2;
  while (ent_slots < 2 * plan.keys.size()) ent_slots <<= 1;
  std::vector<uint32_t> ent_tab(2ull * ent_slots, 0);
  for (const auto& kv : plan.keys) {
    uint32_t at = ent_hash(kv.first) & (ent_slots - 1);
    while (ent_tab[2 * at]) at = (at + 1) & (ent_slots - 1);
    ent_tab[2 * at] = kv.first + 1;
    ent_tab[2 * at + 1] = kv.second | (plan.entry_have_http[kv.second] ? kEntHaveHttp : 0u);
  }
  uint32_t lds_ent_tab = kNone;
  if (!plan.single && 2ull * ent_slots <= kMaxLdsEntWords && img + 2ull * ent_slots <= budget)
    lds_ent_tab = img_take(2ull * ent_slots);
  // candidate-presence bitmasks: one bit per end code; small ones in LDS
  for (uint32_t k = 0; k < ndfa; ++k) {
    const uint64_t words = (ct[k].size() + 31) / 32;
    if (words <= kMaxLdsCtmaskWords && img + words <= budget) dd[k].lds_ctmask = img_take(words);
  }
  auto hotness = [&](uint32_t k) -> int {
    const uint32_t f = all[k].field;
    if (f == kNone) return 0;
    if (f == kFieldPath) return 1;
    if (f == kFieldAuthority) return 2;
    if (f == kFieldMethod) return 3;
    return 4;
  };
  std::vector<uint32_t> order(ndt);
  for (uint32_t k = 0; k < ndt; ++k) order[k] = k;
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return hotness(a) < hotness(b); });
  for (uint32_t k : order) {
    if (dd[k].kind == kDfaAlit || dd[k].lds_table != kNone) continue;  // no automaton / placed above
    if (dd[k].kind == kDfaSearch) {  // walked from the program; the 256-byte class map in LDS when it fits
      if (img + 64 <= budget) dd[k].lds_table = img_take(64);
      // small automata (a method's, a few hosts'): the dense table and its mid
      // masks too, so their steps read LDS instead of L2
      const SearchDfa& sd = all[k].grp->sd;
      const uint64_t tw = sd.table.size();
      if (dd[k].lds_table != kNone && dd[k].lds_mid != kNone && tw <= kLdsSearchMaxWords && img + tw <= budget)
        dd[k].lds_search = img_take(tw);
      continue;
    }
    const PackedDfa& d = *all[k].d;
    const uint64_t half_es = (d.n_slots + 1) / 2, half_latch = (d.latch.size() + 1) / 2;
    const uint64_t need = ((d.n_slots + 3) & ~3ull) + ((half_es + 3) & ~3ull) + ((half_latch + 3) & ~3ull);
    const bool es16 = d.sets.size() < kEs16Latched && all[k].npats < kEs16Latched;
    const bool es8 = d.sets.size() < kEs8Latched && all[k].npats < kEs16Latched;
    if (img + d.n_slots > kLdsTableWords) continue;  // rows are 16-bit byte addresses (program.h)
    const uint64_t need8 = ((d.n_slots + 3) & ~3ull) + ((half_latch + 3) & ~3ull);
    if (es8 && img + need8 <= budget) {  // end codes ride in the slot entries
      dd[k].lds_table = img_take(d.n_slots);
      dd[k].lds_es = kLdsEsInEntry;
      dd[k].lds_latch = 2 * img_take(half_latch);
    } else if (es16 && img + need <= budget) {
      dd[k].lds_table = img_take(d.n_slots);
      dd[k].lds_es = 2 * img_take(half_es);
      dd[k].lds_latch = 2 * img_take(half_latch);
    } else if (img + ((d.n_slots + 3) & ~3ull) <= budget) {
      // the slot table (read once per byte) alone; end codes / latches (read
      // once per walk) stay in the program
      dd[k].lds_table = img_take(d.n_slots);
    }
  }
  // Candidate tables are read once per request (after the walks), so they
  // only go to LDS while the image stays small: record staging space is worth
  // more (measured on MI355X, config 2: 5.0 ms with them in HBM vs 5.5 ms).
  const uint64_t ct_budget = std::min<uint64_t>(budget, kLdsCtBudget / 4);
  for (uint32_t k : order) {
    if (!masks[k].empty() && dd[k].lds_mask == kNone && img + ((2 * masks[k].size() + 3) & ~size_t(3)) <= budget)
      dd[k].lds_mask = img_take(2 * masks[k].size());
  }
  for (uint32_t k : order) {
    if (k < ndfa && img + ((16 * ct[k].size() + 3) & ~size_t(3)) <= ct_budget)
      dd[k].lds_ct = img_take(16 * ct[k].size());
  }

  // literal-anchored patterns' descriptors and literals, last: in LDS when they fit
  // (else program memory)
  std::vector<uint64_t> alit_words(nf, 0);  // AlitRecs (header + literal granules)
  for (uint32_t f = 0; f < nf; ++f)
    for (const auto& L : alit[f].lit) alit_words[f] += 4ull * alit_rec_granules(L.size());
  for (uint32_t f = 0; f < nf; ++f) {
    if (fd[f].alit_tab == kNone) continue;
    const uint64_t words = alit_words[f];
    // (read once per candidate: within the table budget only -- config 2's
    // 1000 path records in LDS shrink the record stage, 32.8 vs 26 ms)
    if (img + words > budget) continue;
    fd[f].alit_lds = 1;
    fd[f].alit_pats = img_take(words);
  }
  // ---- program layout ----
  HttpHeader h;
  std::memset(&h, 0, sizeof h);
  uint64_t w = sizeof(HttpHeader) / 4;
  auto take = [&](uint64_t words) {
    uint64_t o = w;
    w += words;
    return static_cast<uint32_t>(o);
  };
  h.magic = kMagicHttp;
  h.n_rules = static_cast<uint32_t>(n);
  h.n_fields = nf;
  h.n_dfas = ndfa;
  h.always_rule = always_rule;
  h.allow_no_l7 = n == 0 ? 1u : 0u;
  h.has_name_dfa = has_name ? 1u : 0u;
  h.off_dfas = take(static_cast<uint64_t>(ndt) * sizeof(DfaDesc) / 4);
  h.off_fields = take(static_cast<uint64_t>(nf) * sizeof(FieldDesc) / 4);
  h.off_name_field = take(name_field.size());
  h.off_sets = take(sets.size() * 2);
  h.off_remotes = take(static_cast<uint64_t>(n) * 2);
  h.any_remotes = any_remotes ? 1u : 0u;
  h.zero_list = zero_span;
  h.single_entry = plan.single ? 1u : 0u;
  {
    uint64_t m = 0;
    for (uint32_t f = 3; f < nf; ++f) m |= 1ull << std::min<size_t>(field_names[f].size(), 63);
    h.name_len_lo = static_cast<uint32_t>(m);
    h.name_len_hi = static_cast<uint32_t>(m >> 32);
  }
  {
    // DFAs / fields the verification must visit (uniform skips in the kernel)
    uint64_t cm = 0, pm = 0;
    for (uint32_t k = 0; k < ndfa && k < 64; ++k)
      for (const Span& sp : ct[k])
        if (sp.len) {
          cm |= 1ull << k;
          break;
        }
    for (uint32_t f = 0; f < nf; ++f)
      if (fd[f].presence.len) pm |= 1ull << f;
    h.cand_dfas_lo = static_cast<uint32_t>(cm);
    h.cand_dfas_hi = static_cast<uint32_t>(cm >> 32);
    h.pres_fields_lo = static_cast<uint32_t>(pm);
    h.pres_fields_hi = static_cast<uint32_t>(pm >> 32);
  }
  h.n_policies = plan.n_policies;
  h.lds_dcap = lds_dcap;
  // slow path: Span[n_rules] into the pool of (field, program offset) pairs,
  // then the programs
  h.off_slow = kNone;
  h.n_slow = n_slow;
  std::vector<std::vector<uint32_t>> slow_off(nf);
  std::vector<Span> slow_span(n, Span{0, 0});
  if (n_slow) {
    h.off_slow = take(2ull * n);
    for (uint32_t f = 0; f < nf; ++f) {
      slow_off[f].assign(fpats[f].size(), kNone);
      for (size_t pi = 0; pi < fpats[f].size(); ++pi)
        if (!slow_vm[f][pi].empty()) slow_off[f][pi] = take(slow_vm[f][pi].size());
    }
    for (size_t i = 0; i < n; ++i) {
      if (slow_list[i].empty()) continue;
      std::vector<uint32_t> pr;
      for (const auto& fp : slow_list[i]) {
        pr.push_back(fp.first);
        pr.push_back(slow_off[fp.first][fp.second]);
      }
      slow_span[i] = push_list(pr);
      slow_span[i].len /= 2;  // pairs
    }
  }
  for (uint32_t k = 0; k < ndfa; ++k) h.search |= dd[k].kind != kDfaPacked ? 1u : 0u;
  h.ent_mask = ent_slots - 1;
  h.ent_tab_off = take(2ull * ent_slots);
  h.off_pool = take(pool.size());
  h.off_cr = take(cr.size());
  for (uint32_t k = 0; k < ndt; ++k) {
    if (dd[k].kind == kDfaSearch) {
      dd[k].table_off = take(dd[k].n_slots);
      dd[k].es_off = take(dd[k].nstates);  // end masks
      dd[k].latch_off = take(0);
      dd[k].acc_cmap_off = take(256 / 4);
      dd[k].acc_mid_off = take(kSearchMaxMid);
    } else if (dd[k].kind == kDfaAlit) {
      dd[k].table_off = dd[k].es_off = dd[k].latch_off = take(0);
    } else {
      dd[k].table_off = take(all[k].d->n_slots);
      dd[k].es_off = take(all[k].d->n_slots);
      dd[k].latch_off = take(all[k].d->latch.size());
    }
    w = (w + 15) & ~uint64_t(15);  // candidate entries on 64-byte boundaries
    dd[k].ct_off = take(16 * ct[k].size());
    dd[k].ctmask_off = take((ct[k].size() + 31) / 32);
  }
  // Literal values of HBM-walked DFAs (program.h DfaDesc::lit_tab): once such
  // a walk is latched on a literal pattern, the kernel compares the rest of
  // the field with the literal directly (independent loads) instead of one
  // dependent table read per byte.
  std::vector<std::vector<uint32_t>> lit_words(ndt);
  for (uint32_t k = 0; k < ndfa; ++k) {
    if (dd[k].lds_table != kNone || !all[k].grp) continue;
    const Group& g = *all[k].grp;
    bool any = false;
    for (uint32_t l = 0; l < g.pats.size(); ++l) {
      const FieldPattern& fp = fpats[all[k].field][g.pats[l]];
      any |= fp.kind == MatchKind::Value && fp.value.size() >= kLitMinBytes;
    }
    if (!any) continue;
    dd[k].lit_tab = take(2ull * g.pats.size());
    std::vector<uint32_t>& lw = lit_words[k];
    lw.assign(2ull * g.pats.size(), kNone);
    for (uint32_t l = 0; l < g.pats.size(); ++l) {
      const FieldPattern& fp = fpats[all[k].field][g.pats[l]];
      if (fp.kind != MatchKind::Value || fp.value.size() < kLitMinBytes) continue;
      lw[2 * l] = take((fp.value.size() + 3) / 4);
      lw[2 * l + 1] = static_cast<uint32_t>(fp.value.size());
    }
  }
  // literal-anchored patterns' AlitRecs (program memory, 16-byte aligned)
  // when the LDS image has no room for them
  for (uint32_t f = 0; f < nf; ++f) {
    if (fd[f].alit_tab == kNone || fd[f].alit_lds) continue;
    w = (w + 3) & ~uint64_t(3);
    fd[f].alit_pats = take(alit_words[f]);
  }
  w = (w + 63) & ~uint64_t(63);  // 256-byte aligned image
  h.lds_image_off = take(img);
  h.lds_image_words = static_cast<uint32_t>(img);
  h.lds_dfas = lds_dfas;
  h.lds_fields = lds_fields;
  h.lds_name_field = lds_name_field;
  h.lds_name_tab = lds_name_tab;
  h.lds_ent_tab = lds_ent_tab;
  h.name_tab_mask = lds_name_tab != kNone ? name_slots - 1 : 0;
  if (w >= (1ull << 32)) return fail(L7M_ETOOBIG, "program exceeds 16 GiB");
  h.total_words = static_cast<uint32_t>(w);

  std::vector<uint32_t> prog(w, 0);
  uint32_t* P = prog.data();
  uint32_t* I = P + h.lds_image_off;
  uint16_t* I16 = reinterpret_cast<uint16_t*>(I);
  std::memcpy(P, &h, sizeof h);
  for (uint32_t k = 0; k < ndt; ++k) {
    const PackedDfa& d = *all[k].d;
    if (dd[k].kind == kDfaSearch) {
      const SearchDfa& sd = all[k].grp->sd;
      std::memcpy(P + dd[k].table_off, sd.table.data(), sd.table.size() * 4ull);
      std::memcpy(P + dd[k].es_off, sd.endmask.data(), sd.endmask.size() * 4ull);
      std::memcpy(P + dd[k].acc_cmap_off, sd.cmap, 256);
      if (dd[k].lds_table != kNone) std::memcpy(I + dd[k].lds_table, sd.cmap, 256);
      if (dd[k].lds_search != kNone) std::memcpy(I + dd[k].lds_search, sd.table.data(), sd.table.size() * 4ull);
      if (dd[k].lds_mid != kNone) std::memcpy(I + dd[k].lds_mid, sd.midmask.data(), sd.midmask.size() * 4ull);
      std::memcpy(P + dd[k].acc_mid_off, sd.midmask.data(), sd.midmask.size() * 4ull);
    } else {
      std::memcpy(P + dd[k].table_off, d.table.data(), d.n_slots * 4ull);
      std::memcpy(P + dd[k].es_off, d.es.data(), d.n_slots * 4ull);
      std::memcpy(P + dd[k].latch_off, d.latch.data(), d.latch.size() * 4ull);
    }
    std::vector<CandEntry> ce(ct[k].size());
    std::memset(ce.data(), 0, ce.size() * sizeof(CandEntry));
    for (size_t i = 0; i < ct[k].size(); ++i) {
      const Span sp = ct[k][i];
      ce[i].len = sp.len;
      ce[i].off = sp.off;
      if (sp.len) {
        const uint32_t nm = cr_matchers(cr[sp.off + 1]);
        const uint32_t words = 2 + 2 * std::min(nm, kCandInlineMatchers);
        std::memcpy(ce[i].rec, cr.data() + sp.off, words * 4);
        P[dd[k].ctmask_off + i / 32] |= 1u << (i % 32);
        if (dd[k].lds_ctmask != kNone) I[dd[k].lds_ctmask + i / 32] |= 1u << (i % 32);
      }
    }
    if (!ce.empty()) std::memcpy(P + dd[k].ct_off, ce.data(), ce.size() * sizeof(CandEntry));
    if (dd[k].lit_tab != kNone) {
      const std::vector<uint32_t>& lw = lit_words[k];
      std::memcpy(P + dd[k].lit_tab, lw.data(), lw.size() * 4);
      for (uint32_t l = 0; l < all[k].npats; ++l)
        if (lw[2 * l] != kNone) {
          const std::string& v = fpats[all[k].field][all[k].grp->pats[l]].value;
          std::memcpy(P + lw[2 * l], v.data(), v.size());
        }
    }
    if (dd[k].lds_table != kNone) {
      // the LDS copy names rows by image byte address (program.h
      // kLdsRowShift), with the target state's end code when it fits 8 bits
      const uint32_t t0 = dd[k].lds_table;
      const bool in_entry = dd[k].lds_es == kLdsEsInEntry;
      auto es8 = [&](uint32_t base) -> uint32_t {
        return d.es[base] == kLatchedAccept ? kEs8Latched : d.es[base];
      };
      for (uint32_t s = 0; s < d.n_slots; ++s) {
        const uint32_t e = d.table[s], next = e >> 8;
        I[t0 + s] = next ? ((4 * (t0 + next)) << kLdsRowShift) | (in_entry ? es8(next) << 8 : 0u) | (e & 0xffu) : 0u;
      }
      if (in_entry && d.start_base) dd[k].start_es8 = es8(d.start_base);
      for (uint32_t s = 0; dd[k].lds_es != kNone && !in_entry && s < d.n_slots; ++s)
        I16[dd[k].lds_es + s] = d.es[s] == kLatchedAccept ? static_cast<uint16_t>(kEs16Latched)
                                                           : static_cast<uint16_t>(d.es[s]);
      for (size_t s = 0; dd[k].lds_latch != kNone && s < d.latch.size(); ++s)
        I16[dd[k].lds_latch + s] = d.latch[s] == kNone ? static_cast<uint16_t>(kEs16Latched)
                                                        : static_cast<uint16_t>(d.latch[s]);
    }
    if (dd[k].lds_ct != kNone) std::memcpy(I + dd[k].lds_ct, ce.data(), ce.size() * sizeof(CandEntry));
    if (dd[k].lds_mask != kNone) std::memcpy(I + dd[k].lds_mask, masks[k].data(), masks[k].size() * 8);
  }
  std::memcpy(P + h.off_dfas, dd.data(), dd.size() * sizeof(DfaDesc));
  std::memcpy(I + lds_dfas, dd.data(), dd.size() * sizeof(DfaDesc));
  for (size_t k = 0; k < dcaps.size(); ++k) {
    const re::DcapForm& F = dcaps[k].form;
    DcapSpec sp;
    std::memset(&sp, 0, sizeof sp);
    sp.lens = static_cast<uint32_t>(F.p1.size()) | static_cast<uint32_t>(F.l2.size()) << 16;
    sp.min = static_cast<uint32_t>(F.min);
    sp.max = F.max < 0 ? kNone : static_cast<uint32_t>(F.max);
    sp.rdfa = dcap_rdfa[k];
    for (int b = 0; b < 256; ++b)
      if (F.cls.test(b)) sp.cls[b >> 5] |= 1u << (b & 31);
    sp.p1 = dcap_p1[k];
    sp.l2 = dcap_l2[k];
    std::memcpy(I + lds_dcap + 16 * k, &sp, sizeof sp);
    std::memcpy(I + dcap_p1[k], F.p1.data(), F.p1.size());
    std::memcpy(I + dcap_l2[k], F.l2.data(), F.l2.size());
  }
  for (uint32_t f = 0; f < nf; ++f)
    if (fd[f].gram_tab != kNone) std::memcpy(I + fd[f].gram_tab, gram[f].tab.data(), gram[f].tab.size() * 4ull);
  for (uint32_t f = 0; f < nf; ++f) {
    if (fd[f].alit_tab == kNone) continue;
    const AlitField& A = alit[f];
    std::vector<uint32_t> gran(A.pats.size());  // pattern -> its AlitRec's granule
    uint32_t g = 0;
    for (size_t i = 0; i < A.pats.size(); ++i) {
      gran[i] = g;
      g += alit_rec_granules(A.lit[i].size());
    }
    fd[f].alit_granules = g;
    std::vector<uint32_t> tab = A.tab;  // {gram, pattern + 1} -> {gram, granule + 1}
    for (size_t e = 1; e < tab.size(); e += 2)
      if (tab[e]) tab[e] = gran[tab[e] - 1] + 1;
    std::memcpy(I + fd[f].alit_tab, tab.data(), tab.size() * 4ull);
    uint32_t* bloom = I + fd[f].alit_tab - kAlitBloomWords;
    for (size_t e = 0; kAlitBloomWords && e < tab.size(); e += 2)
      if (tab[e + 1]) {
        const uint32_t b = alit_bloom_bit(gram_bucket(tab[e]));
        bloom[b >> 5] |= 1u << (b & 31u);
      }
    uint32_t* base = (fd[f].alit_lds ? I : P) + fd[f].alit_pats;
    for (size_t i = 0; i < A.pats.size(); ++i) {
      const auto loc = fp_loc[f][A.pats[i]];  // (group, local id)
      AlitRec ar;
      ar.len_k = static_cast<uint32_t>(A.lit[i].size()) | A.k[i] << 16;
      ar.code = (dfa_first[f] + loc.first) << 8 | loc.second;
      ar.resid = A.resid[i];
      ar.pad = 0;
      std::memcpy(base + 4 * gran[i], &ar, sizeof ar);
      std::memcpy(reinterpret_cast<uint8_t*>(base + 4 * gran[i] + 4), A.lit[i].data(), A.lit[i].size());
    }
  }
  std::memcpy(P + h.off_fields, fd.data(), fd.size() * sizeof(FieldDesc));
  std::memcpy(I + lds_fields, fd.data(), fd.size() * sizeof(FieldDesc));
  if (lds_name_tab != kNone) {
    for (uint32_t f = 3; f < nf; ++f) {
      const std::string& nm = field_names[f];
      const uint32_t hk = name_hash(nm);
      uint32_t at = hk & (name_slots - 1);
      while (I[lds_name_tab + 4 * at] != 0) at = (at + 1) & (name_slots - 1);
      uint32_t* sl = I + lds_name_tab + 4 * at;
      sl[0] = hk;
      sl[1] = static_cast<uint32_t>(nm.size());
      sl[2] = f;
      sl[3] = name_off[f - 3];
      std::memcpy(I + name_off[f - 3], nm.data(), nm.size());
    }
  }
  std::memcpy(P + h.ent_tab_off, ent_tab.data(), ent_tab.size() * 4);
  if (lds_ent_tab != kNone) std::memcpy(I + lds_ent_tab, ent_tab.data(), ent_tab.size() * 4);
  if (!name_field.empty()) {
    std::memcpy(P + h.off_name_field, name_field.data(), name_field.size() * 4);
    std::memcpy(I + lds_name_field, name_field.data(), name_field.size() * 4);
  }
  std::memcpy(P + h.off_sets, sets.data(), sets.size() * sizeof(Span));
  if (n) std::memcpy(P + h.off_remotes, rremote.data(), rremote.size() * sizeof(Span));
  if (!pool.empty()) std::memcpy(P + h.off_pool, pool.data(), pool.size() * 4);
  if (!cr.empty()) std::memcpy(P + h.off_cr, cr.data(), cr.size() * 4);
  if (n_slow) {
    Span* sl = reinterpret_cast<Span*>(P + h.off_slow);
    for (uint32_t f = 0; f < nf; ++f)
      for (size_t pi = 0; pi < fpats[f].size(); ++pi)
        if (slow_off[f][pi] != kNone)
          std::memcpy(P + slow_off[f][pi], slow_vm[f][pi].data(), slow_vm[f][pi].size() * 4);
    for (size_t i = 0; i < n; ++i) sl[i] = slow_span[i];
  }

  res.program = std::move(prog);
  res.info.proto = L7M_PROTO_HTTP;
  res.info.n_rules = static_cast<uint32_t>(n);
  res.info.n_fields = nf;
  res.info.n_dfas = ndt;
  res.info.total_dfa_states = total_states;
  res.info.program_bytes = static_cast<uint64_t>(w) * 4;
  res.info.n_counters = static_cast<uint32_t>(n) + 2;
  return res;
}

// compile_http_core, and again without the literal-anchored scan of each
// field whose bucket table did not fit the LDS budget (at most once per field).
CompileResult compile_http_alit_fallback(const l7m_http_rule* rules, size_t n, const PolicyPlan& plan,
                                         const l7m_opts& opts) {
  uint64_t no_alit = 0;
  for (;;) {
    uint32_t over = kNone;
    CompileResult r = compile_http_core(rules, n, plan, opts, no_alit, &over);
    if (r.status != L7M_ETOOBIG || over == kNone || over >= 64 || (no_alit >> over & 1)) return r;
    no_alit |= 1ull << over;
  }
}

}  // namespace

CompileResult compile_http(const l7m_http_rule* rules, size_t n, const l7m_opts& opts) {
  // one policy whose every port and direction use `rules`
  PolicyPlan plan;
  plan.single = true;
  plan.n_policies = 1;
  plan.rule_entry.assign(n, 0);
  plan.entry_have_http = {static_cast<uint8_t>(n > 0 ? 1 : 0)};
  plan.names = {""};
  plan.origin.resize(n);
  for (size_t i = 0; i < n; ++i) plan.origin[i] = {0, 1, 0, 0, static_cast<int32_t>(i), 0};
  CompileResult r = compile_http_alit_fallback(rules, n, plan, opts);
  r.names = std::move(plan.names);
  r.origin = std::move(plan.origin);
  return r;
}

// NetworkPolicyMap construction (envoy/cilium_network_policy.h:40-208,
// .cc:42-108) flattened for the kernel: every HTTP rule (or matcher-less
// pseudo rule of a port rule without http_rules) gets an index in the order
// l7m_rule_origin documents and the port entry it belongs to; the
// (policy, direction, port) -> entry table drives the exact-port / port-0 /
// no-entry selection of PortNetworkPolicy::Matches (h:169-192).
CompileResult compile_http_policies(const l7m_network_policy* pols, size_t npol, const l7m_opts& opts) {
  CompileResult bad;
  auto fail = [&](int st, const std::string& m) {
    bad.status = st;
    bad.err = m;
    return bad;
  };
  if (npol > 0 && !pols) return fail(L7M_EINVAL, "policies == NULL");
  if (npol >= L7M_POLICY_UNKNOWN) return fail(L7M_ETOOBIG, "more than 65534 endpoint policies");
  PolicyPlan plan;
  plan.single = false;
  plan.n_policies = static_cast<uint32_t>(npol);
  std::vector<l7m_http_rule> flat;
  std::vector<std::vector<uint32_t>> flat_remotes;  // owned copies
  std::vector<std::string> seen_names;
  for (size_t pi = 0; pi < npol; ++pi) {
    const l7m_network_policy& P = pols[pi];
    const std::string name = P.name ? P.name : "";
    if (std::find(plan.names.begin(), plan.names.end(), name) != plan.names.end())
      return fail(L7M_EINVAL_RULE, "duplicate endpoint policy name '" + name + "'");
    plan.names.push_back(name);
    for (uint32_t dir = 0; dir < 2; ++dir) {
      const uint32_t ingress = dir == 0 ? 1u : 0u;  // ingress, then egress
      const l7m_port_policy* pp = ingress ? P.ingress : P.egress;
      const size_t npp = ingress ? P.n_ingress : P.n_egress;
      if (npp && !pp) return fail(L7M_EINVAL, "port policies == NULL");
      // port entries in input order, the port-0 entry last
      std::vector<size_t> order;
      std::vector<uint32_t> ports_seen;
      for (size_t k = 0; k < npp; ++k) {
        if (pp[k].port > 65535) return fail(L7M_EINVAL_RULE, "port > 65535");
        if (pp[k].protocol != L7M_L4_TCP) continue;  // "NOT installing non-TCP policy" (h:163-165)
        if (std::find(ports_seen.begin(), ports_seen.end(), pp[k].port) != ports_seen.end())
          return fail(L7M_EINVAL_RULE, "PortNetworkPolicy: Duplicate port number " + std::to_string(pp[k].port));
        ports_seen.push_back(pp[k].port);
        if (pp[k].port != 0) order.push_back(k);
      }
      for (size_t k = 0; k < npp; ++k)
        if (pp[k].port == 0 && pp[k].protocol == L7M_L4_TCP) order.push_back(k);
      for (size_t k : order) {
        const l7m_port_policy& E = pp[k];
        if (E.n_rules && !E.rules) return fail(L7M_EINVAL, "port rules == NULL");
        const uint32_t entry = static_cast<uint32_t>(plan.entry_have_http.size());
        if (entry >= kCrMaxEntries) return fail(L7M_ETOOBIG, "too many port entries");
        bool have_http = false;
        for (size_t r = 0; r < E.n_rules; ++r) {
          const l7m_port_rule& R = E.rules[r];
          if (R.n_remote_ids && !R.remote_ids) return fail(L7M_EINVAL, "remote_ids == NULL");
          std::vector<uint32_t> rem(R.remote_ids, R.remote_ids + R.n_remote_ids);
          if (R.has_http_rules) {
            have_http = true;
            if (R.n_http_rules == 0 || !R.http_rules)
              return fail(L7M_EINVAL_RULE, "http_rules present but empty (HttpNetworkPolicyRules min_items = 1)");
            for (size_t j = 0; j < R.n_http_rules; ++j) {
              if (R.http_rules[j].n_remote_ids)
                return fail(L7M_EINVAL, "remote ids belong to the port rule, not to its http rules");
              flat.push_back(R.http_rules[j]);
              flat_remotes.push_back(rem);
              plan.rule_entry.push_back(entry);
              plan.origin.push_back({static_cast<uint32_t>(pi), ingress, E.port, static_cast<uint32_t>(r),
                                     static_cast<int32_t>(j), 0});
            }
          } else {
            flat.push_back(l7m_http_rule{});  // no L7 predicate: any request
            flat_remotes.push_back(rem);
            plan.rule_entry.push_back(entry);
            plan.origin.push_back({static_cast<uint32_t>(pi), ingress, E.port, static_cast<uint32_t>(r), -1, 0});
          }
        }
        plan.entry_have_http.push_back(have_http ? 1 : 0);
        plan.keys.emplace_back(ent_key(static_cast<uint32_t>(pi), ingress, E.port), entry);
      }
    }
  }
  for (size_t i = 0; i < flat.size(); ++i) {
    flat[i].remote_ids = flat_remotes[i].data();
    flat[i].n_remote_ids = static_cast<uint32_t>(flat_remotes[i].size());
  }
  CompileResult r = compile_http_alit_fallback(flat.data(), flat.size(), plan, opts);
  r.names = std::move(plan.names);
  r.origin = std::move(plan.origin);
  return r;
}

}  // namespace l7m
