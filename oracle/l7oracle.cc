// l7oracle.cc — CPU ORACLE for the L7 verdict path.  TEST INFRASTRUCTURE ONLY.
//
// This is a plain restatement of the reference algorithm, used by tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.  The
// product (libl7match.so) never links, loads or calls it.
//
// HTTP (dialect envoy-ecma-full; dialect re2-search replaces regex_match by
// std::regex_search, which equals Go regexp MatchString on the grammar and
// inputs the RE2 tests use — printable ASCII subjects, no CR/LF, no
// engine-specific syntax — pinned by tests/golden/re2_search.json):
//   getHTTPRule            pkg/envoy/server.go:261-320
//   SortHeaderMatchers     pkg/envoy/sort.go:205-250 (panic on nil Regex -> error)
//   HeaderData / matchHeaders (Envoy @ envoy/WORKSPACE:10, called from
//                          envoy/cilium_network_policy.h:68-71): lower-cased name,
//                          first header with that name, std::regex_match for
//                          regex (ECMAScript | optimize, the engine Envoy links),
//                          == for literal values, presence otherwise.
//   OR over rules          envoy/cilium_network_policy.h:98-105 (first index reported)
//   no HTTP rules -> allow envoy/cilium_network_policy.h:129-135
//   NPDS policy maps       PolicyOracle: PortNetworkPolicyRule / PortNetworkPolicyRules /
//                          PortNetworkPolicy / PolicyInstance / NetworkPolicyMap::Allowed
//                          envoy/cilium_network_policy.h:76-237 (exact port, port 0,
//                          no entry -> allow; unknown endpoint policy -> deny)
// Kafka:
//   Sanitize               pkg/policy/api/rule_validation.go:190-233,
//                          MapRoleToAPIKey pkg/policy/api/kafka.go:274-293
//   ReadReq / ReadRequest  vendor/github.com/optiopay/kafka/proto/messages.go:124-165,
//                          pkg/kafka/request.go:186-229 and the per-kind readers
//                          (messages.go:357-482, 493-522, 752-809, 1018-1039,
//                          1158-1213, 1374-1411, 1572-1628, 1791-1839),
//                          decoder semantics serialization.go:30-196, utils.go:9-24
//   compressed sets        messages.go:441-478: gzip (Go compress/gzip framing restated,
//                          DEFLATE by zlib), snappy (github.com/golang/snappy decode.go,
//                          proto/snappy.go), decoded sets read recursively
//   MatchesRule            pkg/kafka/policy.go:27-225
// Regex engines: std::regex (the reference engine, default) or the
// Thompson-NFA / Pike-VM simulator of nfa.h (engine 1, the long-input oracle
// of SURVEY.md §8(c): the same membership, linear time, no recursion; pinned
// against std::regex by tests/cpp/fuzz_nfa.cc).  With engine 1 each pattern is
// still compiled by std::regex too, so NACK parity (L7M_EINVAL_REGEX) is the
// reference's.
// Verdict encoding matches include/l7match.h (-1 deny, i >= 0 deciding rule).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <regex>
#include <set>
#include <unordered_map>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include <pthread.h>
#include <sys/mman.h>
#include <unistd.h>
#include <zlib.h>

#include "../include/l7match.h"
#include "nfa.h"

namespace {

void set_err(char* err, size_t errlen, const std::string& m) {
  if (!err || !errlen) return;
  size_t k = m.size() < errlen - 1 ? m.size() : errlen - 1;
  memcpy(err, m.data(), k);
  err[k] = 0;
}
std::string S(const char* p) { return p ? std::string(p) : std::string(); }

// ============================================================== HTTP ====
struct Matcher {
  std::string name, value;
  bool has_regex;  // Regex != nil
};
struct HeaderData {
  std::string lname;
  uint32_t name_id = 0;  // HttpOracle::name_ids (single rule-list oracle)
  int kind;  // 0 regex, 1 value, 2 present
  std::string value;
  std::regex re;
  std::shared_ptr<const nfa::Prog> nfa;  // engine 1
};

// regex_match / regex_search of a kind-0 matcher with the selected engine
bool regex_ok(const HeaderData& hd, const std::string& v, bool search) {
  if (hd.nfa) {
    thread_local nfa::Runner run;
    return run.run(*hd.nfa, reinterpret_cast<const uint8_t*>(v.data()), v.size(), search);
  }
  return search ? std::regex_search(v, hd.re) : std::regex_match(v, hd.re);
}
// Per-rule prefilter of the linear scan (a necessary condition, so the
// verdicts are unchanged): the rule's first two matchers' header names (ids)
// and the bytes their values must start with -- a literal value's first
// bytes, or a full-match regex's forced prefix (nfa.h forced_prefix).  Kept
// in one contiguous array so rejecting a rule touches one cache line instead
// of the rule's std::regex / NFA objects (config 5: 100k rules per request).
struct RulePre {
  uint32_t nid[2];
  uint8_t len[2];
  uint8_t n;           // matchers described (0..2)
  uint8_t has_remote;  // allowed_remotes_ non-empty
  char b[2][12];
};
struct HttpOracle {
  bool search = false;  // L7M_DIALECT_RE2_SEARCH
  std::vector<std::vector<HeaderData>> rules;
  std::vector<std::unordered_set<uint32_t>> remotes;  // allowed_remotes_ (empty = any)
  std::unordered_map<std::string, uint32_t> name_ids;  // lower-cased header names of the rules
  std::vector<RulePre> pre;
  bool prefilter = true;  // orc_http_set_prefilter(h, 0): the plain scan (bench.py's cpu_baseline)
};

bool hm_less(const Matcher& a, const Matcher& b) {
  if (a.name != b.name) return a.name < b.name;
  if (a.value != b.value) return a.value < b.value;
  return !a.has_regex && b.has_regex;  // only reached for regex/regex pairs
}

// Parsed record view.
struct HttpReq {
  bool ok = false;
  std::vector<std::pair<std::string, std::string>> headers;  // pseudo first
  uint32_t remote_id = 0;
  uint32_t dport = 0, policy = 0;
  bool ingress = false;
};

HttpReq parse_http(const uint8_t* arena, size_t arena_bytes, uint64_t off) {
  HttpReq q;
  if ((off & 3) || off + L7M_HTTP_REC_FIXED > arena_bytes) return q;
  const uint8_t* r = arena + off;
  uint32_t w[5];
  memcpy(w, r, sizeof w);
  uint32_t len = w[0], flags = (w[2] >> 16) & 0xff, nh = w[2] >> 24;
  uint32_t ml = w[3] & 0xffff, pl = w[3] >> 16, al = w[4] & 0xffff;
  if (off + ((uint64_t(len) + 3) & ~3ull) > arena_bytes) return q;
  uint64_t need = L7M_HTTP_REC_FIXED + 4ull * nh + ml + pl + al;
  if (need > len) return q;
  std::vector<std::pair<uint32_t, uint32_t>> dir(nh);
  for (uint32_t j = 0; j < nh; ++j) {
    uint32_t e;
    memcpy(&e, r + L7M_HTTP_REC_FIXED + 4 * j, 4);
    dir[j] = {e & 0xffff, e >> 16};
    need += dir[j].first + dir[j].second;
  }
  if (need != len) return q;
  q.remote_id = w[1];
  q.dport = w[2] & 0xffff;
  q.ingress = (flags & L7M_HTTP_F_INGRESS) != 0;
  q.policy = w[4] >> 16;
  size_t p = L7M_HTTP_REC_FIXED + 4ull * nh;
  auto take = [&](uint32_t l) {
    std::string s(reinterpret_cast<const char*>(r + p), l);
    p += l;
    return s;
  };
  std::string m = take(ml), pa = take(pl), au = take(al);
  if (flags & L7M_HTTP_F_METHOD) q.headers.push_back({":method", m});
  if (flags & L7M_HTTP_F_PATH) q.headers.push_back({":path", pa});
  if (flags & L7M_HTTP_F_AUTHORITY) q.headers.push_back({":authority", au});
  for (auto& d : dir) {
    std::string n = take(d.first), v = take(d.second);
    if (!n.empty() && n[0] == ':') continue;  // record contract: no pseudo names here
    q.headers.push_back({n, v});
  }
  q.ok = true;
  return q;
}

int32_t eval_http_one(const HttpOracle& o, const HttpReq& q) {
  if (!q.ok) return L7M_VERDICT_PARSE_ERROR;
  if (o.rules.empty()) return L7M_VERDICT_ALLOW_NO_L7;
  // the request's value of each header name the rules use (first occurrence,
  // as Envoy's HeaderMap::get)
  thread_local std::vector<const std::string*> vals;
  vals.assign(o.name_ids.size(), nullptr);
  for (const auto& h : q.headers) {
    auto it = o.name_ids.find(h.first);
    if (it != o.name_ids.end() && !vals[it->second]) vals[it->second] = &h.second;
  }
  for (size_t i = 0; i < o.rules.size(); ++i) {
    const RulePre& pr = o.pre[i];
    bool cand = true;
    for (uint32_t k = 0; o.prefilter && k < pr.n && cand; ++k) {
      const std::string* v = vals[pr.nid[k]];
      cand = v && v->size() >= pr.len[k] && std::memcmp(v->data(), pr.b[k], pr.len[k]) == 0;
    }
    if (!cand) continue;
    // PortNetworkPolicyRule::Matches: remote id first (cilium_network_policy.h:90-97)
    if (pr.has_remote && !o.remotes[i].count(q.remote_id)) continue;
    bool all = true;
    for (const auto& hd : o.rules[i]) {
      const std::string* v = vals[hd.name_id];
      if (!v) { all = false; break; }
      if (hd.kind == 0 && !regex_ok(hd, *v, o.search)) {
        all = false;
        break;
      }
      if (hd.kind == 1 && *v != hd.value) { all = false; break; }
    }
    if (all) return static_cast<int32_t>(i);
  }
  return L7M_VERDICT_DENY;
}

// ============================================================= Kafka ====
// getHTTPRule (pkg/envoy/server.go:261-320) + SortHeaderMatchers
// (pkg/envoy/sort.go:205-250) + Envoy HeaderData construction.
int build_http_rule(const l7m_http_rule& r, std::vector<HeaderData>* out, std::string* err, int engine) {
  std::vector<Matcher> ms;
  if (!S(r.path).empty()) ms.push_back({":path", S(r.path), true});
  if (!S(r.method).empty()) ms.push_back({":method", S(r.method), true});
  if (!S(r.host).empty()) ms.push_back({":authority", S(r.host), true});
  for (uint32_t j = 0; j < r.n_headers; ++j) {
    std::string h = S(r.headers[j]);
    size_t sp = h.find(' ');
    if (sp != std::string::npos) {
      std::string k = h.substr(0, sp);
      while (!k.empty() && k.back() == ':') k.pop_back();
      ms.push_back({k, h.substr(sp + 1), false});
    } else {
      ms.push_back({h, "", false});
    }
  }
  for (size_t a = 0; a < ms.size(); ++a)
    for (size_t b = a + 1; b < ms.size(); ++b)
      if (ms[a].name == ms[b].name && ms[a].value == ms[b].value && !(ms[a].has_regex && ms[b].has_regex)) {
        *err = "sort panic: duplicate header matcher";
        return L7M_EINVAL_RULE;
      }
  std::sort(ms.begin(), ms.end(), hm_less);
  for (auto& m : ms) {
    if (m.name.empty()) {
      *err = "empty header name";
      return L7M_EINVAL_RULE;
    }
    HeaderData hd;
    hd.lname = m.name;
    for (auto& c : hd.lname) c = (char)tolower((unsigned char)c);
    hd.value = m.value;
    if (m.value.empty()) hd.kind = 2;
    else if (m.has_regex) {
      hd.kind = 0;
      try {
        hd.re = std::regex(m.value, std::regex::optimize);
      } catch (const std::regex_error& e) {
        *err = std::string("regex: ") + e.what();
        return L7M_EINVAL_REGEX;
      }
      if (engine == 1) {
        try {
          hd.nfa = std::make_shared<const nfa::Prog>(nfa::compile(m.value));
        } catch (const nfa::Unsupported& e) {
          *err = std::string("nfa oracle: ") + e.what();
          return L7M_EUNSUPPORTED;
        } catch (const nfa::SyntaxError& e) {  // std::regex accepted it: the two parsers disagree
          *err = std::string("nfa oracle parser disagrees with std::regex: ") + e.what();
          return L7M_EUNSUPPORTED;
        }
      }
    } else hd.kind = 1;
    out->push_back(std::move(hd));
  }
  return L7M_OK;
}

// ConfigUtility::matchHeaders (HttpNetworkPolicyRule::Matches, h:68-71).
bool match_headers(const std::vector<HeaderData>& hds, const HttpReq& q, bool search) {
  for (const auto& hd : hds) {
    const std::string* v = nullptr;
    for (const auto& h : q.headers)
      if (h.first == hd.lname) {
        v = &h.second;
        break;
      }
    if (!v) return false;
    if (hd.kind == 0 && !regex_ok(hd, *v, search)) return false;
    if (hd.kind == 1 && *v != hd.value) return false;
  }
  return true;
}

struct OPortRule {  // PortNetworkPolicyRule (h:76-112)
  std::unordered_set<uint32_t> remotes;
  std::vector<std::vector<HeaderData>> http;
  int32_t base = 0;  // flattened index of its first HTTP rule
  // Matches (h:90-108): the deciding index, or -1
  int32_t matches(uint32_t remote_id, const HttpReq& q, bool search) const {
    if (!remotes.empty() && !remotes.count(remote_id)) return -1;
    if (!http.empty()) {
      for (size_t j = 0; j < http.size(); ++j)
        if (match_headers(http[j], q, search)) return base + static_cast<int32_t>(j);
      return -1;
    }
    return base;  // empty set matches any payload
  }
};
struct OPortRules {  // PortNetworkPolicyRules (h:114-150)
  std::vector<OPortRule> rules;
  bool have_http = false;
  int32_t matches(uint32_t remote_id, const HttpReq& q, bool search) const {
    if (!have_http) return L7M_VERDICT_ALLOW_NO_L7;
    if (rules.empty()) return L7M_VERDICT_ALLOW_NO_L7;
    for (const auto& r : rules) {
      const int32_t v = r.matches(remote_id, q, search);
      if (v >= 0) return v;
    }
    return -1;
  }
};
struct OPolicy {  // PolicyInstance (h:40-208)
  std::unordered_map<uint32_t, OPortRules> ingress, egress;
};
struct PolicyOracle {  // NetworkPolicyMap
  bool search = false;
  std::map<std::string, uint32_t> names;
  std::vector<OPolicy> pols;
};

// PortNetworkPolicy::Matches (h:169-192) under NetworkPolicyMap::Allowed
// (h:223-237; the record carries the endpoint policy's index).
int32_t eval_policy_one(const PolicyOracle& o, const HttpReq& q) {
  if (!q.ok) return L7M_VERDICT_PARSE_ERROR;
  if (q.policy >= o.pols.size()) return L7M_VERDICT_DENY;  // no policy for the endpoint
  const auto& m = q.ingress ? o.pols[q.policy].ingress : o.pols[q.policy].egress;
  bool found = false;
  auto it = m.find(q.dport);
  if (it != m.end()) {
    const int32_t v = it->second.matches(q.remote_id, q, o.search);
    if (v >= 0) return v;
    found = true;
  }
  it = m.find(0);
  if (it != m.end()) {
    const int32_t v = it->second.matches(q.remote_id, q, o.search);
    if (v >= 0) return v;
    found = true;
  }
  return found ? L7M_VERDICT_DENY : L7M_VERDICT_ALLOW_NO_PORT_POLICY;
}


struct KRule {
  std::vector<int16_t> keys;  // apiKeyInt
  bool has_version = false;
  int16_t version = 0;
  std::string client, topic;
};
struct KafkaOracle {
  std::vector<KRule> rules;
  // L7DataMap (pkg/policy/l4.go:110-129): rule i belongs to entry group[i];
  // a source's relevant entries are those whose selector matches it plus the
  // wildcard entries.  !selective: one wildcard entry, every rule applies.
  std::vector<uint32_t> group;
  bool selective = false;
  uint64_t wild = ~0ull;
  std::map<uint32_t, uint64_t> id_mask;
  uint64_t mask_of(uint32_t identity) const {
    if (!selective) return ~0ull;
    auto it = identity ? id_mask.find(identity) : id_mask.end();
    return it == id_mask.end() ? wild : it->second;  // nil identity: wildcard entries only
  }
};

const std::map<std::string, int16_t>& api_key_map() {
  static const std::map<std::string, int16_t> m = {
      {"produce", 0}, {"fetch", 1}, {"offsets", 2}, {"metadata", 3}, {"leaderandisr", 4},
      {"stopreplica", 5}, {"updatemetadata", 6}, {"controlledshutdown", 7}, {"offsetcommit", 8},
      {"offsetfetch", 9}, {"findcoordinator", 10}, {"joingroup", 11}, {"heartbeat", 12},
      {"leavegroup", 13}, {"syncgroup", 14}, {"describegroups", 15}, {"listgroups", 16},
      {"saslhandshake", 17}, {"apiversions", 18}, {"createtopics", 19}, {"deletetopics", 20},
      {"deleterecords", 21}, {"initproducerid", 22}, {"offsetforleaderepoch", 23},
      {"addpartitionstotxn", 24}, {"addoffsetstotxn", 25}, {"endtxn", 26},
      {"writetxnmarkers", 27}, {"txnoffsetcommit", 28}, {"describeacls", 29},
      {"createacls", 30}, {"deleteacls", 31}, {"describeconfigs", 32}, {"alterconfigs", 33}};
  return m;
}

// Go strings.ToLower for the inputs that can matter here: ASCII, plus the two
// non-ASCII runes that lower-case to ASCII (U+0130 -> 'i', U+212A -> 'k').
std::string go_lower(const std::string& s) {
  std::string r;
  for (size_t i = 0; i < s.size();) {
    unsigned char c = s[i];
    if (c == 0xC4 && i + 1 < s.size() && (unsigned char)s[i + 1] == 0xB0) { r += 'i'; i += 2; continue; }
    if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x84 && (unsigned char)s[i + 2] == 0xAA) {
      r += 'k'; i += 3; continue;
    }
    r += (c >= 'A' && c <= 'Z') ? char(c - 'A' + 'a') : char(c);
    ++i;
  }
  return r;
}

// strconv.ParseInt(s, 10, 16)
bool go_parse_int16(const std::string& s, int16_t* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
  if (i >= s.size()) return false;
  long long v = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
    if (v > 40000) v = 40000;
  }
  if (neg) v = -v;
  if (v < -32768 || v > 32767) return false;
  *out = static_cast<int16_t>(v);
  return true;
}

bool topic_chars_ok(const std::string& t) {  // ^[a-zA-Z0-9\\._\\-]+$ (Go regexp)
  if (t.empty()) return false;
  for (unsigned char c : t) {
    bool ok = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') ||
              c == '\\' || c == '.' || c == '_' || c == '-';
    if (!ok) return false;
  }
  return true;
}

int sanitize(const l7m_kafka_rule& in, KRule* r, std::string* err) {
  std::string role = S(in.role), key = S(in.api_key), ver = S(in.api_version);
  r->client = S(in.client_id);
  r->topic = S(in.topic);
  if (!key.empty() && !role.empty()) { *err = "Cannot set both Role and APIKey together"; return L7M_EINVAL_RULE; }
  if (!key.empty()) {
    auto it = api_key_map().find(go_lower(key));
    if (it == api_key_map().end()) { *err = "invalid Kafka APIKey"; return L7M_EINVAL_RULE; }
    r->keys.push_back(it->second);
  }
  if (!role.empty()) {
    std::string lr = go_lower(role);
    if (lr == "produce") r->keys = {0, 3, 18};
    else if (lr == "consume") r->keys = {1, 2, 3, 8, 9, 10, 11, 12, 13, 14, 18};
    else { *err = "invalid Kafka APIRole"; return L7M_EINVAL_RULE; }
  }
  if (!ver.empty()) {
    if (!go_parse_int16(ver, &r->version)) { *err = "invalid Kafka APIVersion"; return L7M_EINVAL_RULE; }
    r->has_version = true;
  }
  if (!r->topic.empty()) {
    if (r->topic.size() > 255) { *err = "kafka topic exceeds maximum len of 255"; return L7M_EINVAL_RULE; }
    if (!topic_chars_ok(r->topic)) { *err = "invalid Kafka Topic name"; return L7M_EINVAL_RULE; }
  }
  return L7M_OK;
}

// ---- decoder with the optiopay error semantics --------------------------
const int64_t kMaxParseBuf = 100LL * 65535;  // maxParseBufSize

struct Reader {  // bytes.Reader / LimitReader view over a byte range
  const uint8_t* p;
  size_t len, pos = 0;
  size_t avail() const { return len - pos; }
};

struct Dec {
  Reader* r;
  bool err = false;
  bool read(uint8_t* out, size_t n) {  // io.ReadFull
    if (r->avail() < n) {
      r->pos = r->len;  // ReadFull consumes what is there before failing
      return false;
    }
    if (out) memcpy(out, r->p + r->pos, n);
    r->pos += n;
    return true;
  }
  int64_t be(size_t n) {
    if (err) return 0;
    uint8_t b[8];
    if (!read(b, n)) { err = true; return 0; }
    uint64_t v = 0;
    for (size_t i = 0; i < n; ++i) v = (v << 8) | b[i];
    if (n == 1) return (int8_t)v;
    if (n == 2) return (int16_t)v;
    if (n == 4) return (int32_t)v;
    return (int64_t)v;
  }
  int8_t i8() { return (int8_t)be(1); }
  int16_t i16() { return (int16_t)be(2); }
  int32_t i32() { return (int32_t)be(4); }
  int64_t i64() { return be(8); }
  uint32_t u32() { return (uint32_t)be(4); }
  std::string str() {
    if (err) return "";
    int16_t n = i16();
    if (err || n < 1) return "";
    std::string s(n, '\0');
    if (!read(reinterpret_cast<uint8_t*>(&s[0]), n)) { err = true; return ""; }
    return s;
  }
  // DecodeBytes; *alloc_err set when allocParseBuf fails
  bool bytes(std::string* out) {
    if (err) return false;
    int32_t n = i32();
    if (err || n < 1) return false;
    if (n > kMaxParseBuf) { err = true; return false; }
    std::string s(n, '\0');
    if (!read(reinterpret_cast<uint8_t*>(&s[0]), n)) { err = true; return false; }
    if (out) *out = s;
    return true;
  }
  // DecodeArrayLen: returns false on ErrInvalidArrayLen
  bool arraylen(int64_t* n) {
    int32_t v = i32();
    if (v < 0 || v > kMaxParseBuf) return false;
    *n = v;
    return true;
  }
};

uint32_t crc32_ieee(const uint8_t* p, size_t n) {
  static uint32_t tbl[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      tbl[i] = c;
    }
    init = true;
  }
  uint32_t c = 0xffffffffu;
  for (size_t i = 0; i < n; ++i) c = tbl[(c ^ p[i]) & 0xff] ^ (c >> 8);
  return c ^ 0xffffffffu;
}

enum MsRc { MS_OK, MS_ERR, MS_UNSUPPORTED };

// ---- compressed message sets (messages.go:441-478) -------------------------
// gzip.NewReader + ioutil.ReadAll (Go compress/gzip, multistream): the member
// framing restated here, the DEFLATE data inflated by zlib (raw mode) — an
// implementation independent of the product's device decoder.  A decoded
// size above maxParseBufSize fails readMessageSet's size check, so inflating
// stops there with an error.  Returns true on success.
bool go_gunzip(const std::string& in, std::vector<uint8_t>* out) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(in.data());
  const size_t n = in.size();
  size_t pos = 0;
  auto header = [&]() -> int {  // 0 ok, 1 error, 2 io.EOF
    const size_t rem = n - pos;
    if (rem == 0) return 2;                                        // ReadFull: EOF
    if (rem < 10) return 1;                                        // ErrUnexpectedEOF
    if (p[pos] != 0x1f || p[pos + 1] != 0x8b || p[pos + 2] != 8) return 1;  // ErrHeader
    const uint8_t flg = p[pos + 3];
    size_t q = pos + 10;
    if (flg & 0x04) {  // FEXTRA
      if (n - q < 2) return 1;
      const size_t xl = p[q] | (p[q + 1] << 8);
      q += 2;
      if (n - q < xl) return 1;
      q += xl;
    }
    for (int f : {0x08, 0x10}) {  // FNAME, FCOMMENT (readString: z.buf is 512 bytes)
      if (!(flg & f)) continue;
      for (int i = 0;; ++i) {
        if (i >= 512) return 1;
        if (q >= n) return 2;  // ReadByte's io.EOF is returned as is
        if (p[q++] == 0) break;
      }
    }
    if (flg & 0x02) {  // FHCRC
      if (n - q < 2) return 1;
      const uint32_t c = static_cast<uint32_t>(crc32(0L, p + pos, static_cast<uInt>(q - pos)));
      if ((p[q] | (p[q + 1] << 8)) != (c & 0xffff)) return 1;
      q += 2;
    }
    pos = q;
    return 0;
  };
  if (header() != 0) return false;  // NewReader fails, io.EOF included
  for (;;) {
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, -15) != Z_OK) return false;
    zs.next_in = const_cast<Bytef*>(p + pos);
    zs.avail_in = static_cast<uInt>(n - pos);
    const size_t start = out->size();
    std::vector<uint8_t> buf(1 << 16);
    int rc;
    do {
      zs.next_out = buf.data();
      zs.avail_out = static_cast<uInt>(buf.size());
      rc = inflate(&zs, Z_NO_FLUSH);
      out->insert(out->end(), buf.data(), buf.data() + (buf.size() - zs.avail_out));
      if (out->size() > static_cast<size_t>(kMaxParseBuf)) rc = Z_DATA_ERROR;
    } while (rc == Z_OK);
    const size_t left = zs.avail_in;
    inflateEnd(&zs);
    if (rc != Z_STREAM_END) return false;
    pos = n - left;
    if (n - pos < 8) return false;
    const uint32_t c = static_cast<uint32_t>(crc32(0L, out->data() + start, static_cast<uInt>(out->size() - start)));
    const uint32_t wc = p[pos] | (p[pos + 1] << 8) | (p[pos + 2] << 16) | ((uint32_t)p[pos + 3] << 24);
    const uint32_t wl = p[pos + 4] | (p[pos + 5] << 8) | (p[pos + 6] << 16) | ((uint32_t)p[pos + 7] << 24);
    if (c != wc || static_cast<uint32_t>(out->size() - start) != wl) return false;  // ErrChecksum
    pos += 8;
    const int h = header();
    if (h == 2) return true;
    if (h == 1) return false;
  }
}

// github.com/golang/snappy Decode (decode.go:25-72, decode_other.go:14-102).
bool go_snappy_block(const uint8_t* src, size_t n, std::vector<uint8_t>* out) {
  uint64_t v = 0;
  unsigned shift = 0;
  size_t hl = 0;
  for (size_t i = 0;; ++i) {  // binary.Uvarint
    if (i >= n) return false;
    const uint8_t b = src[i];
    if (b < 0x80) {
      if (i > 9 || (i == 9 && b > 1)) return false;
      v |= (uint64_t)b << shift;
      hl = i + 1;
      break;
    }
    v |= (uint64_t)(b & 0x7f) << shift;
    shift += 7;
  }
  if (v > 0xffffffffull) return false;
  if (out->size() + v > static_cast<uint64_t>(kMaxParseBuf)) return false;  // the set cannot pass readMessageSet
  const size_t base = out->size();
  out->resize(base + v);
  uint8_t* dst = out->data() + base;
  const int64_t dlen = (int64_t)v;
  int64_t d = 0, s = (int64_t)hl, len = (int64_t)n, length = 0, offset = 0;
  while (s < len) {
    const int tag = src[s] & 3;
    if (tag == 0) {
      uint32_t x = src[s] >> 2;
      if (x < 60) {
        s++;
      } else {
        const int k = (int)x - 59;
        s += 1 + k;
        if (s > len) return false;
        x = 0;
        for (int i = 0; i < k; ++i) x |= (uint32_t)src[s - k + i] << (8 * i);
      }
      length = (int64_t)x + 1;
      if (length > dlen - d || length > len - s) return false;
      memcpy(dst + d, src + s, (size_t)length);
      d += length;
      s += length;
      continue;
    } else if (tag == 1) {
      s += 2;
      if (s > len) return false;
      length = 4 + ((src[s - 2] >> 2) & 7);
      offset = ((src[s - 2] & 0xe0) << 3) | src[s - 1];
    } else if (tag == 2) {
      s += 3;
      if (s > len) return false;
      length = 1 + (src[s - 3] >> 2);
      offset = src[s - 2] | (src[s - 1] << 8);
    } else {
      s += 5;
      if (s > len) return false;
      length = 1 + (src[s - 5] >> 2);
      offset = (int64_t)((uint32_t)src[s - 4] | ((uint32_t)src[s - 3] << 8) | ((uint32_t)src[s - 2] << 16) |
                         ((uint32_t)src[s - 1] << 24));
    }
    if (offset <= 0 || d < offset || length > dlen - d) return false;
    for (int64_t end = d + length; d != end; ++d) dst[d] = dst[d - offset];
  }
  return d == dlen;
}

// proto/snappy.go snappyDecode; its out-of-range slicing on short snappy-java
// framing panics in the reference — reported here as an error.
bool go_snappy(const std::string& in, std::vector<uint8_t>* out) {
  const uint8_t* b = reinterpret_cast<const uint8_t*>(in.data());
  const size_t n = in.size();
  static const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
  if (n < 8 || memcmp(b, magic, 8) != 0) return go_snappy_block(b, n, out);
  if (n < 12) return false;
  const uint32_t ver = ((uint32_t)b[8] << 24) | (b[9] << 16) | (b[10] << 8) | b[11];
  if (ver != 1) return false;
  for (size_t i = 16; i < n;) {
    if (n - i < 4) return false;
    const size_t cl = ((uint32_t)b[i] << 24) | (b[i + 1] << 16) | (b[i + 2] << 8) | b[i + 3];
    i += 4;
    if (cl > n - i) return false;
    if (!go_snappy_block(b + i, cl, out)) return false;
    i += cl;
  }
  return true;
}

// readMessageSet(r, size, version): reads at most `size` bytes of `outer`,
// decompressing gzip / snappy messages and reading their sets recursively.
MsRc read_message_set(Reader* outer, int32_t size, int16_t version) {
  if (size < 0 || size > kMaxParseBuf) return MS_ERR;
  size_t lim = outer->avail() < (size_t)size ? outer->avail() : (size_t)size;
  Reader rd{outer->p + outer->pos, lim, 0};
  auto done = [&]() { outer->pos += rd.pos; };
  Dec dec{&rd};
  for (;;) {
    dec.i64();
    if (dec.err) { done(); return MS_OK; }   // EOF / ErrUnexpectedEOF
    int32_t msz = dec.i32();
    if (dec.err) { done(); return MS_OK; }
    if (msz <= 0) { done(); return MS_OK; }
    if (msz > kMaxParseBuf) { done(); return MS_ERR; }
    if (rd.avail() < (size_t)msz) { rd.pos = rd.len; done(); return MS_OK; }
    const uint8_t* mb = rd.p + rd.pos;
    rd.pos += msz;
    Reader mr{mb, (size_t)msz, 0};
    Dec md{&mr};
    uint32_t crc = md.u32();
    if (msz <= 4) { done(); return MS_OK; }
    if (crc != crc32_ieee(mb + 4, msz - 4)) { done(); return MS_OK; }
    md.i8();
    int8_t attr = md.i8();
    if (version >= 1) md.i64();
    int comp = attr & 3;
    if (comp == 0) {
      md.bytes(nullptr);
      md.bytes(nullptr);
      if (md.err) { done(); return MS_ERR; }
    } else if (comp == 1 || comp == 2) {
      md.bytes(nullptr);  // key ignored
      std::string val;
      md.bytes(&val);     // nil for a length < 1
      if (md.err) { done(); return MS_ERR; }
      std::vector<uint8_t> decoded;
      const bool ok = comp == 1 ? go_gunzip(val, &decoded) : go_snappy(val, &decoded);
      if (!ok || decoded.size() > (size_t)kMaxParseBuf) { done(); return MS_ERR; }
      Reader in{decoded.data(), decoded.size(), 0};
      if (read_message_set(&in, (int32_t)decoded.size(), version) == MS_ERR) { done(); return MS_ERR; }
    } else {
      done();
      return MS_OK;  // `return nil, err` with err == nil (messages.go:479-480)
    }
  }
}

struct KReq {
  int32_t status = 0;  // 0 ok, PARSE_ERROR, UNSUPPORTED
  int16_t kind = 0, version = 0;
  int type = 0;  // 0 nil request, 1 typed (client + topics), 2 ConsumerMetadata
  std::string client;
  std::vector<std::string> topics;
};

KReq parse_kafka(const uint8_t* arena, size_t arena_bytes, uint64_t off) {
  KReq q;
  q.status = L7M_VERDICT_PARSE_ERROR;
  if (off + 4 > arena_bytes) return q;
  const uint8_t* r = arena + off;
  int32_t msize = (int32_t)((uint32_t)r[0] << 24 | (uint32_t)r[1] << 16 | (uint32_t)r[2] << 8 | r[3]);
  if (msize <= 0) return q;                         // io.ErrUnexpectedEOF
  if (msize < 2) return q;                          // kind: short read
  if ((int64_t)msize + 4 > kMaxParseBuf) return q;  // allocParseBuf
  if (off + 4 + (uint64_t)msize > arena_bytes) return q;
  size_t blen = 4 + (size_t)msize;
  if (blen < 12) return q;  // "unexpected end of request"
  q.kind = (int16_t)((r[4] << 8) | r[5]);
  q.version = (int16_t)((r[6] << 8) | r[7]);
  Reader rd{r, blen, 0};
  Dec d{&rd};
  d.i32();
  d.i16();
  int16_t ver = d.i16();
  d.i32();
  int k = q.kind;
  if (k != 0 && k != 1 && k != 2 && k != 3 && k != 8 && k != 9 && k != 10) {
    q.type = 0;
    q.status = 0;
    return q;
  }
  q.client = d.str();
  q.type = (k == 10) ? 2 : 1;
  int64_t n;
  auto topic_list = [&](auto&& per_topic) -> bool {
    if (!d.arraylen(&n)) return false;
    for (int64_t t = 0; t < n; ++t) {
      q.topics.push_back(d.str());
      if (!per_topic()) return false;
      if (d.err) {  // remaining iterations are no-ops; the final Err() check fails
        return true;
      }
    }
    return true;
  };
  bool ok = true;
  MsRc ms = MS_OK;
  switch (k) {
    case 0:  // Produce
      if (ver >= 3) d.str();
      d.i16();
      d.i32();
      ok = topic_list([&]() {
        int64_t np;
        if (!d.arraylen(&np)) return false;
        for (int64_t p = 0; p < np; ++p) {
          d.i32();
          if (d.err) return false;
          int32_t mss = d.i32();
          if (d.err) return false;
          MsRc rc = read_message_set(&rd, mss, ver);
          if (rc == MS_ERR) return false;
          if (rc == MS_UNSUPPORTED) { ms = MS_UNSUPPORTED; return false; }
        }
        return true;
      });
      break;
    case 1:  // Fetch
      d.i32();
      d.i32();
      d.i32();
      if (ver >= 3) d.i32();
      if (ver >= 4) d.i8();
      ok = topic_list([&]() {
        int64_t np;
        if (!d.arraylen(&np)) return false;
        for (int64_t p = 0; p < np && !d.err; ++p) {
          d.i32();
          d.i64();
          if (ver >= 5) d.i64();
          d.i32();
        }
        return true;
      });
      break;
    case 2:  // Offset
      d.i32();
      if (ver >= 2) d.i8();
      ok = topic_list([&]() {
        int64_t np;
        if (!d.arraylen(&np)) return false;
        for (int64_t p = 0; p < np && !d.err; ++p) {
          d.i32();
          d.i64();
          if (ver == 0) d.i32();
        }
        return true;
      });
      break;
    case 3:  // Metadata
      ok = topic_list([&]() { return true; });
      if (ok && ver >= 4) d.i8();
      break;
    case 8:  // OffsetCommit
      d.str();
      if (ver >= 1) { d.i32(); d.str(); }
      if (ver >= 2) d.i64();
      ok = topic_list([&]() {
        int64_t np;
        if (!d.arraylen(&np)) return false;
        for (int64_t p = 0; p < np && !d.err; ++p) {
          d.i32();
          d.i64();
          if (ver == 1) d.i64();
          d.str();
        }
        return true;
      });
      break;
    case 9:  // OffsetFetch
      d.str();
      ok = topic_list([&]() {
        int64_t np;
        if (!d.arraylen(&np)) return false;
        for (int64_t p = 0; p < np && !d.err; ++p) d.i32();
        return true;
      });
      break;
    case 10:  // ConsumerMetadata
      d.str();
      if (ver >= 1) d.i8();
      break;
  }
  if (ms == MS_UNSUPPORTED) { q.status = L7M_VERDICT_UNSUPPORTED; return q; }
  if (!ok || d.err) { q.status = L7M_VERDICT_PARSE_ERROR; return q; }
  if (k == 10) q.topics.clear();  // GetTopics: nil for ConsumerMetadata
  q.status = 0;
  return q;
}

bool is_topic_api_key(int16_t k) {
  switch (k) {
    case 0: case 1: case 2: case 3: case 4: case 5: case 6: case 8: case 9: case 19: case 20:
    case 21: case 23: case 24: case 27: case 28: case 34: case 35: case 37:
      return true;
  }
  return false;
}

bool rule_matches(const KReq& q, const KRule& r) {
  if (!r.keys.empty()) {
    bool hit = false;
    for (int16_t k : r.keys) hit |= k == q.kind;
    if (!hit) return false;
  }
  if (r.has_version && r.version != q.version) return false;
  if (r.topic.empty() && r.client.empty()) return true;
  if (q.type == 1) return r.client.empty() || r.client == q.client;
  if (q.type == 2) return true;
  return !(!r.topic.empty() && is_topic_api_key(q.kind));
}

// MatchesRule (policy.go:197-225) over GetRelevantRules' list: the rules
// that apply to the source (mask), in compiled order.
int32_t eval_kafka_one(const KafkaOracle& o, const KReq& q, uint64_t mask = ~0ull) {
  if (q.status) return q.status;
  std::set<std::string> left(q.topics.begin(), q.topics.end());
  for (size_t i = 0; i < o.rules.size(); ++i) {
    if (o.selective && !((mask >> o.group[i]) & 1)) continue;
    const KRule& r = o.rules[i];
    if (r.topic.empty() || q.topics.empty()) {
      if (rule_matches(q, r)) return (int32_t)i;
    } else if (left.count(r.topic)) {
      if (rule_matches(q, r)) {
        left.erase(r.topic);
        if (left.empty()) return (int32_t)i;
      }
    }
  }
  return L7M_VERDICT_DENY;
}

// Run f() on a fresh thread whose 1 GiB stack is reserved but not committed,
// and report how many bytes of it were touched (mincore: the lowest resident
// page).  That is the native stack the reference engine's recursion needs for
// this call -- std::regex_match overflows an Envoy worker's 8 MiB default
// stack exactly when it exceeds that.
template <class F>
uint64_t run_on_measured_stack(F&& f) {
  const size_t sz = 1ull << 30, pg = static_cast<size_t>(sysconf(_SC_PAGESIZE));
  void* stk = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (stk == MAP_FAILED) return ~0ull;
  struct Job {
    F* f;
    static void* run(void* p) {
      (*static_cast<Job*>(p)->f)();
      return nullptr;
    }
  } job{&f};
  pthread_attr_t at;
  pthread_attr_init(&at);
  pthread_attr_setstack(&at, stk, sz);
  pthread_t t;
  uint64_t used = ~0ull;
  if (pthread_create(&t, &at, &Job::run, &job) == 0) {
    pthread_join(t, nullptr);
    std::vector<unsigned char> res(sz / pg);
    if (mincore(stk, sz, res.data()) == 0) {
      size_t lo = res.size();
      for (size_t k = 0; k < res.size(); ++k)
        if (res[k] & 1) {
          lo = k;
          break;
        }
      used = static_cast<uint64_t>(res.size() - lo) * pg;
    }
  }
  pthread_attr_destroy(&at);
  munmap(stk, sz);
  return used;
}

template <class F>
void parallel_for(size_t n, int threads, F&& f) {
  if (threads <= 1 || n < 2 * static_cast<size_t>(threads)) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t]() {
      size_t a = n * t / threads, b = n * (t + 1) / threads;
      for (size_t i = a; i < b; ++i) f(i);
    });
  for (auto& x : th) x.join();
}

}  // namespace

extern "C" {

int orc_http_new_engine(const l7m_http_rule* rules, size_t n, uint32_t dialect, int engine, void** out, char* err,
                        size_t errlen) {
  auto* o = new HttpOracle();
  o->search = dialect == L7M_DIALECT_RE2_SEARCH;
  for (size_t i = 0; i < n; ++i) {
    std::vector<HeaderData> hds;
    std::string e;
    int rc = build_http_rule(rules[i], &hds, &e, engine);
    if (rc) {
      set_err(err, errlen, e);
      delete o;
      return rc;
    }
    RulePre pr{};
    for (auto& hd : hds) {
      auto it = o->name_ids.emplace(hd.lname, static_cast<uint32_t>(o->name_ids.size())).first;
      hd.name_id = it->second;
      if (pr.n == 2) continue;
      std::string pfx;
      if (hd.kind == 1) {
        pfx = hd.value;
      } else if (hd.kind == 0 && !o->search) {
        try {
          pfx = nfa::compile(hd.value).prefix;
        } catch (const std::exception&) {  // outside nfa.h's subset: no prefilter bytes
        }
      }
      if (pfx.size() > sizeof pr.b[0]) pfx.resize(sizeof pr.b[0]);
      pr.nid[pr.n] = hd.name_id;
      pr.len[pr.n] = static_cast<uint8_t>(pfx.size());
      std::memcpy(pr.b[pr.n], pfx.data(), pfx.size());
      ++pr.n;
    }
    pr.has_remote = rules[i].n_remote_ids != 0;
    o->pre.push_back(pr);
    o->rules.push_back(std::move(hds));
    std::unordered_set<uint32_t> rem;
    for (uint32_t j = 0; j < rules[i].n_remote_ids; ++j) rem.insert(rules[i].remote_ids[j]);
    o->remotes.push_back(std::move(rem));
  }
  *out = o;
  return L7M_OK;
}

int orc_http_new_dialect(const l7m_http_rule* rules, size_t n, uint32_t dialect, void** out, char* err,
                         size_t errlen) {
  return orc_http_new_engine(rules, n, dialect, 0, out, err, errlen);
}

// NetworkPolicyMap restated (envoy/cilium_network_policy.h:40-237,
// npds.proto:32-118).  Verdict index = the flattened position of the deciding
// HTTP rule in the order include/l7match.h (l7m_rule_origin) documents.
int orc_http_policies_new_engine(const l7m_network_policy* pols, size_t n, uint32_t dialect, int engine, void** out,
                                 char* err, size_t errlen) {
  auto* o = new PolicyOracle();
  o->search = dialect == L7M_DIALECT_RE2_SEARCH;
  int32_t index = 0;
  for (size_t pi = 0; pi < n; ++pi) {
    const l7m_network_policy& P = pols[pi];
    OPolicy op;
    for (int dir = 0; dir < 2; ++dir) {
      const l7m_port_policy* pp = dir == 0 ? P.ingress : P.egress;
      const size_t npp = dir == 0 ? P.n_ingress : P.n_egress;
      auto& m = dir == 0 ? op.ingress : op.egress;
      // index order: port entries as given, the port-0 entry last
      std::vector<size_t> order;
      for (size_t k = 0; k < npp; ++k)
        if (pp[k].port != 0) order.push_back(k);
      for (size_t k = 0; k < npp; ++k)
        if (pp[k].port == 0) order.push_back(k);
      for (size_t k : order) {
        if (pp[k].protocol != L7M_L4_TCP) continue;  // h:156-166
        OPortRules prs;
        for (size_t r = 0; r < pp[k].n_rules; ++r) {
          const l7m_port_rule& R = pp[k].rules[r];
          OPortRule pr;
          for (uint32_t j = 0; j < R.n_remote_ids; ++j) pr.remotes.insert(R.remote_ids[j]);
          pr.base = index;
          if (R.has_http_rules) {
            prs.have_http = true;
            if (R.n_http_rules == 0) {
              set_err(err, errlen, "empty http_rules");
              delete o;
              return L7M_EINVAL_RULE;
            }
            for (size_t j = 0; j < R.n_http_rules; ++j) {
              std::vector<HeaderData> hds;
              std::string e;
              int rc = build_http_rule(R.http_rules[j], &hds, &e, engine);
              if (rc) {
                set_err(err, errlen, e);
                delete o;
                return rc;
              }
              pr.http.push_back(std::move(hds));
              ++index;
            }
          } else {
            ++index;
          }
          prs.rules.push_back(std::move(pr));
        }
        if (!m.emplace(pp[k].port, std::move(prs)).second) {
          set_err(err, errlen, "PortNetworkPolicy: Duplicate port number");
          delete o;
          return L7M_EINVAL_RULE;
        }
      }
    }
    o->names.emplace(S(P.name), static_cast<uint32_t>(pi));
    o->pols.push_back(std::move(op));
  }
  *out = o;
  return L7M_OK;
}

int orc_http_policies_new(const l7m_network_policy* pols, size_t n, uint32_t dialect, void** out, char* err,
                          size_t errlen) {
  return orc_http_policies_new_engine(pols, n, dialect, 0, out, err, errlen);
}

int orc_http_policies_eval(void* h, const uint8_t* arena, size_t arena_bytes, const uint64_t* offs, size_t n,
                           int32_t* verdicts, int threads) {
  const PolicyOracle& o = *static_cast<PolicyOracle*>(h);
  parallel_for(n, threads, [&](size_t i) { verdicts[i] = eval_policy_one(o, parse_http(arena, arena_bytes, offs[i])); });
  return L7M_OK;
}

void orc_http_policies_free(void* h) { delete static_cast<PolicyOracle*>(h); }

int orc_http_new(const l7m_http_rule* rules, size_t n, void** out, char* err, size_t errlen) {
  return orc_http_new_dialect(rules, n, L7M_DIALECT_ENVOY_ECMA_FULL, out, err, errlen);
}

int orc_http_eval(void* h, const uint8_t* arena, size_t arena_bytes, const uint64_t* offs, size_t n,
                  int32_t* verdicts, int threads) {
  const HttpOracle& o = *static_cast<HttpOracle*>(h);
  parallel_for(n, threads, [&](size_t i) { verdicts[i] = eval_http_one(o, parse_http(arena, arena_bytes, offs[i])); });
  return L7M_OK;
}

void orc_http_free(void* h) { delete static_cast<HttpOracle*>(h); }

// orc_http_eval one request at a time, each on a measured stack: stack_used[i]
// = native stack bytes the reference's evaluation of request i touched (the
// rules' matchers in index order, as eval_http_one runs them).
int orc_http_eval_stack(void* h, const uint8_t* arena, size_t arena_bytes, const uint64_t* offs, size_t n,
                        int32_t* verdicts, uint64_t* stack_used) {
  const HttpOracle& o = *static_cast<HttpOracle*>(h);
  for (size_t i = 0; i < n; ++i) {
    const HttpReq q = parse_http(arena, arena_bytes, offs[i]);
    int32_t v = L7M_VERDICT_PARSE_ERROR;
    stack_used[i] = run_on_measured_stack([&]() { v = eval_http_one(o, q); });
    verdicts[i] = v;
  }
  return L7M_OK;
}

// std::regex_match(input, pattern) on a measured stack: the result (1 / 0,
// -1 if the pattern does not compile) and the native stack bytes it touched.
int orc_regex_match_stack(const char* pattern, const char* input, size_t input_len, uint64_t* stack_used) {
  int r = -1;
  try {
    std::regex re(pattern, std::regex::ECMAScript | std::regex::optimize);
    const std::string s(input, input_len);
    *stack_used = run_on_measured_stack([&]() { r = std::regex_match(s, re) ? 1 : 0; });
  } catch (const std::regex_error&) {
    r = -1;
  }
  return r;
}

// 0: evaluate every rule's matchers (the reference's per-request loop as
// Envoy runs it), 1 (default): skip rules the per-rule prefilter rejects.
void orc_http_set_prefilter(void* h, int on) { static_cast<HttpOracle*>(h)->prefilter = on != 0; }

int orc_regex_match(const char* pattern, const char* input, size_t input_len) {
  try {
    std::regex re(pattern, std::regex::optimize);
    return std::regex_match(std::string(input, input_len), re) ? 1 : 0;
  } catch (...) {
    return -1;
  }
}

int orc_regex_search(const char* pattern, const char* input, size_t input_len) {
  try {
    std::regex re(pattern, std::regex::optimize);
    return std::regex_search(std::string(input, input_len), re) ? 1 : 0;
  } catch (...) {
    return -1;
  }
}

// The NFA simulator on one pattern: 1 / 0, -1 syntax error, -2 unsupported.
int orc_nfa_match(const char* pattern, const char* input, size_t input_len, int search) {
  try {
    const nfa::Prog p = nfa::compile(pattern);
    nfa::Runner run;
    return run.run(p, reinterpret_cast<const uint8_t*>(input), input_len, search != 0) ? 1 : 0;
  } catch (const nfa::SyntaxError&) {
    return -1;
  } catch (const nfa::Unsupported&) {
    return -2;
  }
}

int orc_kafka_new(const l7m_kafka_rule* rules, size_t n, void** out, char* err, size_t errlen) {
  auto* o = new KafkaOracle();
  for (size_t i = 0; i < n; ++i) {
    KRule r;
    std::string e;
    int rc = sanitize(rules[i], &r, &e);
    if (rc) {
      set_err(err, errlen, "rule " + std::to_string(i) + ": " + e);
      delete o;
      return rc;
    }
    o->rules.push_back(std::move(r));
  }
  *out = o;
  return L7M_OK;
}

int orc_kafka_eval(void* h, const uint8_t* arena, size_t arena_bytes, const uint64_t* offs, size_t n,
                   int32_t* verdicts, int threads) {
  const KafkaOracle& o = *static_cast<KafkaOracle*>(h);
  parallel_for(n, threads, [&](size_t i) { verdicts[i] = eval_kafka_one(o, parse_kafka(arena, arena_bytes, offs[i])); });
  return L7M_OK;
}

// An L7DataMap: entries of (rules, wildcard) and, per source identity, the
// entries whose selector matches it.
int orc_kafka_new_map(const l7m_kafka_selector_rules* map, size_t n_entries, const l7m_identity_selectors* ids,
                      size_t n_ids, void** out, char* err, size_t errlen) {
  auto* o = new KafkaOracle();
  o->wild = 0;
  for (size_t g = 0; g < n_entries; ++g) {
    if (map[g].wildcard) o->wild |= 1ull << g;
    else o->selective = true;
    for (size_t j = 0; j < map[g].n_rules; ++j) {
      KRule r;
      std::string e;
      int rc = sanitize(map[g].rules[j], &r, &e);
      if (rc) {
        set_err(err, errlen, "rule " + std::to_string(o->rules.size()) + ": " + e);
        delete o;
        return rc;
      }
      o->rules.push_back(std::move(r));
      o->group.push_back(static_cast<uint32_t>(g));
    }
  }
  for (size_t k = 0; k < n_ids; ++k) {
    uint64_t m = o->wild;
    for (size_t j = 0; j < ids[k].n_selectors; ++j) m |= 1ull << ids[k].selectors[j];
    o->id_mask[ids[k].identity] = m;
  }
  *out = o;
  return L7M_OK;
}

int orc_kafka_eval_ids(void* h, const uint8_t* arena, size_t arena_bytes, const uint64_t* offs, size_t n,
                       const uint32_t* ids, int32_t* verdicts, int threads) {
  const KafkaOracle& o = *static_cast<KafkaOracle*>(h);
  parallel_for(n, threads, [&](size_t i) {
    verdicts[i] = eval_kafka_one(o, parse_kafka(arena, arena_bytes, offs[i]), o.mask_of(ids ? ids[i] : 0u));
  });
  return L7M_OK;
}

void orc_kafka_free(void* h) { delete static_cast<KafkaOracle*>(h); }

// proto/snappy.go snappyDecode of one value (framed or a bare block), for the
// snappy known-answer tests: 0 decoded (out_len bytes into out), 1 the
// reference returns an error (or panics), 2 out too small.
int orc_snappy_decode(const uint8_t* src, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
  std::vector<uint8_t> d;
  if (!go_snappy(std::string(reinterpret_cast<const char*>(src), n), &d)) return 1;
  if (d.size() > cap) return 2;
  if (!d.empty()) memcpy(out, d.data(), d.size());
  *out_len = d.size();
  return 0;
}

}  // extern "C"
