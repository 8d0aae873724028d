// l7gen.cc — deterministic synthetic rule / request generators for the
// BASELINE.json configurations (libl7gen.so; bench + tests harness, not part
// of the verdict path).  Every request i is generated from
// splitmix64(seed, i) alone, so any shard [start, start + count) of a
// workload is reproducible and independent of how the batch is split across
// GPUs.  Workload shapes follow SURVEY.md §8(d).
//
// Configs:
//   1  README HTTP policy (GET /public/.*, X-Token: [0-9]+), seed 0xC1
//   2  1k HTTP path/method/host/header rules, seed 0xC2
//   3  Kafka topic/clientID/apiKey rules (10k), seed 0xC3
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/l7match.h"

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  uint32_t u(uint32_t n) { return static_cast<uint32_t>(next() % n); }
  bool p(double x) { return (next() >> 11) * (1.0 / 9007199254740992.0) < x; }
};

uint64_t mix(uint64_t seed, uint64_t i) {
  Rng r(seed * 0x100000001b3ull ^ (i + 0x632be59bd9b4e019ull));
  r.next();
  return r.next();
}

std::string digits(Rng& r, int lo, int hi) {
  int n = lo + static_cast<int>(r.u(hi - lo + 1));
  std::string s;
  for (int k = 0; k < n; ++k) s.push_back(static_cast<char>('0' + r.u(10)));
  return s;
}
std::string word(Rng& r, int lo, int hi, const char* alpha = "abcdefghijklmnopqrstuvwxyz") {
  int n = lo + static_cast<int>(r.u(hi - lo + 1));
  size_t m = std::strlen(alpha);
  std::string s;
  for (int k = 0; k < n; ++k) s.push_back(alpha[r.u(static_cast<uint32_t>(m))]);
  return s;
}

// ----------------------------------------------------------------- HTTP --
struct HttpRuleT {
  int method;  // 0 GET, 1 POST, 2 GET|HEAD, 3 PUT|PATCH, 4 [A-Z]+
  bool svc;    // path template /svc{i}/... vs /api/{w}/.*
  std::string w;
  bool host;
  int hdr;     // 0 none, 1 x-tenant literal, 2 x-debug presence
};

const char* kMethods[] = {"GET", "POST", "GET|HEAD", "PUT|PATCH", "[A-Z]+"};

std::vector<HttpRuleT> http_rules_cfg2(uint64_t seed, uint32_t n) {
  std::vector<HttpRuleT> v(n);
  for (uint32_t i = 0; i < n; ++i) {
    Rng r(mix(seed ^ 0x52554c45ull, i));
    v[i].method = static_cast<int>(r.u(5));
    v[i].svc = r.p(0.5);
    v[i].w = word(r, 4, 10);
    v[i].host = r.p(0.3);
    v[i].hdr = r.p(0.2) ? (r.p(0.5) ? 1 : 2) : 0;
  }
  return v;
}

struct Req {
  std::string method, path, authority;
  bool has_auth = true;
  std::vector<std::pair<std::string, std::string>> hdrs;
};

void fillers(Rng& r, Req& q) {
  q.hdrs.push_back({"user-agent", "curl/7." + digits(r, 2, 2) + "." + digits(r, 1, 1)});
  q.hdrs.push_back({"accept", "*/*"});
  if (r.p(0.8)) q.hdrs.push_back({"x-request-id", word(r, 16, 16, "0123456789abcdef")});
}

void mutate(Rng& r, std::string& s) {
  if (s.empty()) return;
  size_t k = r.u(static_cast<uint32_t>(s.size()));
  s[k] = static_cast<char>(0x20 + r.u(0x5f));
}

Req http_req_cfg1(uint64_t seed, uint64_t i) {
  Rng r(mix(seed, i));
  Req q;
  uint32_t m = r.u(10);
  q.method = m < 5 ? "GET" : m < 7 ? "POST" : m < 8 ? "PUT" : m < 9 ? "DELETE" : "HEAD";
  if (r.p(0.5)) {
    q.path = "/public/" + word(r, 0, 48, "abcdefghijklmnopqrstuvwxyz0123456789/");
  } else {
    uint32_t k = r.u(3);
    q.path = k == 0 ? "/private/" + word(r, 0, 32) : k == 1 ? "/api/v1/" + word(r, 0, 32) : "/";
  }
  q.authority = "svc" + digits(r, 1, 2) + ".example.com";
  fillers(r, q);
  if (r.p(0.7)) {
    uint32_t k = r.u(100);
    std::string v = k < 70 ? digits(r, 1, 12) : k < 85 ? "[0-9]+" : word(r, 1, 12);
    q.hdrs.insert(q.hdrs.begin() + r.u(static_cast<uint32_t>(q.hdrs.size() + 1)), {"x-token", v});
  }
  return q;
}

Req http_req_cfg2(const std::vector<HttpRuleT>& rules, uint64_t seed, uint64_t i) {
  Rng r(mix(seed, i));
  uint32_t ri = r.u(static_cast<uint32_t>(rules.size()));
  const HttpRuleT& t = rules[ri];
  Req q;
  static const char* any_m[] = {"GET", "POST", "PUT", "DELETE", "PATCH", "HEAD", "OPTIONS"};
  switch (t.method) {
    case 0: q.method = "GET"; break;
    case 1: q.method = "POST"; break;
    case 2: q.method = r.p(0.5) ? "GET" : "HEAD"; break;
    case 3: q.method = r.p(0.5) ? "PUT" : "PATCH"; break;
    default: q.method = any_m[r.u(7)]; break;
  }
  static const char* res[] = {"users", "orders", "items"};
  if (t.svc) q.path = "/svc" + std::to_string(ri) + "/v" + digits(r, 1, 2) + "/" + res[r.u(3)] + "/" + digits(r, 1, 8);
  else q.path = "/api/" + t.w + "/" + word(r, 0, 24, "abcdefghijklmnopqrstuvwxyz0123456789/._-");
  if (t.host) q.authority = "svc" + std::to_string(ri % 50) + ".ns.local";
  else q.authority = r.p(0.5) ? "svc" + std::to_string(r.u(100)) + ".ns.local" : "example.com";
  fillers(r, q);
  // config 2's mean record is ~150 B; the fillers above give
  // ~128 B, so most requests also carry the accept-encoding header a browser
  // or client library sends (no rule references it)
  static const char* enc[] = {"gzip", "gzip, deflate", "gzip, deflate, br", "br", "identity", "deflate, gzip"};
  if (r.p(0.72)) q.hdrs.push_back({"accept-encoding", enc[r.u(6)]});
  if (t.hdr == 1) q.hdrs.push_back({"x-tenant", "t" + std::to_string(ri % 17)});
  if (t.hdr == 2) q.hdrs.push_back({"x-debug", "1"});
  if (r.p(0.5)) {  // one-byte mutation of a matched field
    uint32_t k = r.u(4);
    if (k == 0) mutate(r, q.method);
    else if (k == 1 || (k == 3 && t.hdr != 1)) mutate(r, q.path);
    else if (k == 2) mutate(r, q.authority);
    else mutate(r, q.hdrs.back().second);
  }
  return q;
}

// ------------------------------------------------------ adversarial (5) --
// NFA-heavy path families and long header values.
//   i % 5 == 0: /a{i}/(a|aa)*b            (alternation blow-up for backtrackers)
//   i % 5 == 1: /x{i}/.*(x|y).*(z|w).*q    (wildcards)
//   i % 5 == 2: /l{i}/(w0|...|w99)          (100-way literal alternation)
//   i % 5 == 3: /c{i}/[a-z]*[a-z]*[a-z]*[a-z]*z
//   i % 5 == 4: /f{i}/(.{0,8}){1,8}foo      (counted-repeat blow-up)
// Every 97th rule also requires the literal header x-blob: <1 KiB value>.
std::string adv_word(uint32_t i, uint32_t k) {
  Rng r(mix(0x574f5244ull ^ i, k));
  return word(r, 3, 8);
}
std::string adv_blob(uint32_t i, uint32_t len) {
  Rng r(mix(0x424c4f42ull, i));
  return word(r, len, len, "abcdefghijklmnopqrstuvwxyz0123456789-_.");
}
std::string adv_path_rule(uint32_t i) {
  const std::string id = std::to_string(i);
  switch (i % 5) {
    case 0: return "/a" + id + "/(a|aa)*b";
    case 1: return "/x" + id + "/.*(x|y).*(z|w).*q";
    case 2: {
      std::string alt;
      for (uint32_t k = 0; k < 100; ++k) alt += (k ? "|" : "") + adv_word(i, k);
      return "/l" + id + "/(" + alt + ")";
    }
    case 3: return "/c" + id + "/[a-z]*[a-z]*[a-z]*[a-z]*z";
    default: return "/f" + id + "/(.{0,8}){1,8}foo";
  }
}
Req http_req_cfg5(uint64_t seed, uint32_t n_rules, uint64_t i) {
  Rng r(mix(seed, i));
  const uint32_t ri = r.u(n_rules);
  const std::string id = std::to_string(ri);
  const bool good = r.p(0.5);
  Req q;
  q.method = "GET";
  switch (ri % 5) {
    case 0: q.path = "/a" + id + "/" + std::string(r.u(21), 'a') + (good ? "b" : "c"); break;
    case 1: q.path = "/x" + id + "/" + word(r, 0, 30, "xyzwq.") + (good ? "q" : "."); break;
    case 2: q.path = "/l" + id + "/" + (good ? adv_word(ri, r.u(100)) : word(r, 3, 8)); break;
    case 3: q.path = "/c" + id + "/" + word(r, 0, 20) + (good ? "z" : "y"); break;
    default: q.path = "/f" + id + "/" + word(r, 0, 70, "abfo.") + (good ? "foo" : "fob"); break;
  }
  q.authority = "adv.example";
  fillers(r, q);
  if (ri % 97 == 0 && r.p(0.8)) {
    std::string b = adv_blob(ri, 1024);
    if (!r.p(0.7)) b[r.u(1024)] = '#';
    q.hdrs.push_back({"x-blob", b});
  } else if (r.p(0.03)) {
    q.hdrs.push_back({"x-blob", adv_blob(static_cast<uint32_t>(i), 1024 + r.u(65535 - 1024))});
  }
  return q;
}

size_t pack(const Req& q, uint8_t* out, uint32_t remote, uint16_t dport) {
  std::vector<const char*> n, v;
  for (auto& h : q.hdrs) {
    n.push_back(h.first.c_str());
    v.push_back(h.second.c_str());
  }
  l7m_http_request x{};
  x.method = q.method.c_str();
  x.path = q.path.c_str();
  x.authority = q.has_auth ? q.authority.c_str() : nullptr;
  x.header_names = n.data();
  x.header_values = v.data();
  x.n_headers = static_cast<uint32_t>(q.hdrs.size());
  x.remote_id = remote;
  x.dport = dport;
  x.ingress = 1;
  // local copy of the record layout (l7m_pack_http lives in libl7match)
  size_t ml = q.method.size(), pl = q.path.size(), al = q.has_auth ? q.authority.size() : 0;
  size_t b = L7M_HTTP_REC_FIXED + 4 * q.hdrs.size() + ml + pl + al;
  for (auto& h : q.hdrs) b += h.first.size() + h.second.size();
  size_t padded = (b + 3) & ~size_t(3);
  if (!out) return padded;
  std::memset(out, 0, padded);
  uint32_t flags = L7M_HTTP_F_METHOD | L7M_HTTP_F_PATH | (q.has_auth ? L7M_HTTP_F_AUTHORITY : 0) | L7M_HTTP_F_INGRESS;
  uint32_t w[5] = {static_cast<uint32_t>(b), remote,
                   static_cast<uint32_t>(dport) | (flags << 16) | (static_cast<uint32_t>(q.hdrs.size()) << 24),
                   static_cast<uint32_t>(ml | (pl << 16)), static_cast<uint32_t>(al)};
  std::memcpy(out, w, sizeof w);
  size_t p = L7M_HTTP_REC_FIXED;
  for (auto& h : q.hdrs) {
    uint32_t e = static_cast<uint32_t>(h.first.size() | (h.second.size() << 16));
    std::memcpy(out + p, &e, 4);
    p += 4;
  }
  auto put = [&](const std::string& s) {
    std::memcpy(out + p, s.data(), s.size());
    p += s.size();
  };
  put(q.method);
  put(q.path);
  if (q.has_auth) put(q.authority);
  for (auto& h : q.hdrs) {
    put(h.first);
    put(h.second);
  }
  (void)x;
  return padded;
}

// ---------------------------------------------------------------- Kafka --
struct KRuleT {
  int keymode;  // 0 apiKey produce, 1 apiKey fetch, 2 role produce, 3 role consume
  bool client;
  int version;  // -1 none
};
std::vector<KRuleT> kafka_rules_cfg3(uint64_t seed, uint32_t n) {
  std::vector<KRuleT> v(n);
  for (uint32_t i = 0; i < n; ++i) {
    Rng r(mix(seed ^ 0x4b52554cull, i));
    v[i].keymode = static_cast<int>(r.u(4));
    v[i].client = r.p(0.5);
    v[i].version = r.p(0.2) ? static_cast<int>(r.u(6)) : -1;
  }
  return v;
}

struct Wire {
  std::vector<uint8_t> b;
  void u8(uint8_t x) { b.push_back(x); }
  void i16(int16_t x) { b.push_back(uint8_t(uint16_t(x) >> 8)); b.push_back(uint8_t(x)); }
  void i32(int32_t x) { for (int k = 3; k >= 0; --k) b.push_back(uint8_t(uint32_t(x) >> (8 * k))); }
  void i64(int64_t x) { for (int k = 7; k >= 0; --k) b.push_back(uint8_t(uint64_t(x) >> (8 * k))); }
  void str(const std::string& s) { i16(static_cast<int16_t>(s.size())); b.insert(b.end(), s.begin(), s.end()); }
};

// Request encoders following the optiopay readers (messages.go) field order.
std::vector<uint8_t> kafka_req_cfg3(uint64_t seed, uint64_t i) {
  Rng r(mix(seed, i));
  uint32_t kk = r.u(3);
  int16_t kind = kk == 0 ? 0 : kk == 1 ? 1 : 3;
  int16_t ver = kind == 0 ? int16_t(r.u(4)) : kind == 1 ? int16_t(r.u(6)) : int16_t(r.u(5));
  std::string client = "client-" + std::to_string(r.u(120));
  uint32_t nt = 1 + r.u(4);
  std::vector<std::string> topics;
  for (uint32_t t = 0; t < nt; ++t) topics.push_back("topic-" + std::to_string(r.u(12000)));
  Wire w;
  w.i32(0);
  w.i16(kind);
  w.i16(ver);
  w.i32(static_cast<int32_t>(r.u(1u << 30)));
  w.str(client);
  if (kind == 0) {
    if (ver >= 3) w.i16(-1);  // null transactional id
    w.i16(1);
    w.i32(1000);
    w.i32(static_cast<int32_t>(nt));
    for (auto& t : topics) {
      w.str(t);
      w.i32(1);
      w.i32(static_cast<int32_t>(r.u(8)));
      w.i32(0);  // empty message set
    }
  } else if (kind == 1) {
    w.i32(-1);
    w.i32(500);
    w.i32(1);
    if (ver >= 3) w.i32(1 << 20);
    if (ver >= 4) w.u8(0);
    w.i32(static_cast<int32_t>(nt));
    for (auto& t : topics) {
      w.str(t);
      w.i32(1);
      w.i32(static_cast<int32_t>(r.u(8)));
      w.i64(static_cast<int64_t>(r.u(1u << 30)));
      if (ver >= 5) w.i64(0);
      w.i32(1 << 20);
    }
  } else {
    if (r.p(0.1)) nt = 0, topics.clear();
    w.i32(static_cast<int32_t>(topics.size()));
    for (auto& t : topics) w.str(t);
    if (ver >= 4) w.u8(1);
  }
  uint32_t sz = static_cast<uint32_t>(w.b.size() - 4);
  w.b[0] = uint8_t(sz >> 24);
  w.b[1] = uint8_t(sz >> 16);
  w.b[2] = uint8_t(sz >> 8);
  w.b[3] = uint8_t(sz);
  return w.b;
}

template <class F>
void parallel(uint64_t count, int threads, F&& f) {
  if (threads <= 1 || count < 4096) {
    f(0, count);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t]() { f(count * t / threads, count * (t + 1) / threads); });
  for (auto& x : th) x.join();
}

std::string g_text;

}  // namespace

extern "C" {

// Rules as text: one rule per line, fields separated by \t:
//   HTTP : path \t method \t host \t header1 \x1f header2 ...
//   Kafka: role \t apiKey \t apiVersion \t clientID \t topic
// Returns a pointer valid until the next call (not thread-safe).
const char* l7g_rules_text(int config, uint64_t seed, uint32_t n_rules) {
  g_text.clear();
  if (config == 1) {
    g_text = "/public/.*\tGET\t\tX-Token: [0-9]+\n";
  } else if (config == 2) {
    auto rules = http_rules_cfg2(seed, n_rules);
    for (uint32_t i = 0; i < n_rules; ++i) {
      const auto& t = rules[i];
      std::string path = t.svc ? "/svc" + std::to_string(i) + "/v[0-9]+/(users|orders|items)/[0-9]+"
                               : "/api/" + t.w + "/.*";
      std::string host = t.host ? "svc" + std::to_string(i % 50) + "\\.ns\\.local" : "";
      std::string hdr = t.hdr == 1 ? "x-tenant: t" + std::to_string(i % 17) : t.hdr == 2 ? "x-debug" : "";
      g_text += path + "\t" + kMethods[t.method] + "\t" + host + "\t" + hdr + "\n";
    }
  } else if (config == 5) {
    for (uint32_t i = 0; i < n_rules; ++i) {
      g_text += adv_path_rule(i) + "\tGET\t\t";
      if (i % 97 == 0) g_text += "x-blob: " + adv_blob(i, 1024);
      g_text += "\n";
    }
  } else if (config == 3) {
    auto rules = kafka_rules_cfg3(seed, n_rules);
    for (uint32_t i = 0; i < n_rules; ++i) {
      const auto& t = rules[i];
      std::string role = t.keymode == 2 ? "produce" : t.keymode == 3 ? "consume" : "";
      std::string key = t.keymode == 0 ? "produce" : t.keymode == 1 ? "fetch" : "";
      std::string ver = t.version >= 0 ? std::to_string(t.version) : "";
      std::string client = t.client ? "client-" + std::to_string(i % 100) : "";
      g_text += role + "\t" + key + "\t" + ver + "\t" + client + "\ttopic-" + std::to_string(i) + "\n";
    }
  }
  return g_text.c_str();
}

// Generate requests [start, start + count) of `config` into arena/offsets
// (offsets relative to arena).  Pass arena == NULL to get the byte size.
// Returns bytes used, or 0 if cap is too small.
uint64_t l7g_requests(int config, uint64_t seed, uint32_t n_rules, uint64_t start, uint64_t count,
                      uint8_t* arena, uint64_t cap, uint64_t* offsets, int threads) {
  std::vector<HttpRuleT> h2;
  if (config == 2) h2 = http_rules_cfg2(seed, n_rules);
  auto gen_one = [&](uint64_t i, uint8_t* out) -> size_t {
    if (config == 1) return pack(http_req_cfg1(seed, i), out, 1, 80);
    if (config == 2) return pack(http_req_cfg2(h2, seed, i), out, 1, 80);
    if (config == 5) return pack(http_req_cfg5(seed, n_rules, i), out, 1, 80);
    auto w = kafka_req_cfg3(seed, i);
    size_t padded = (w.size() + 3) & ~size_t(3);
    if (out) {
      std::memset(out, 0, padded);
      std::memcpy(out, w.data(), w.size());
    }
    return padded;
  };
  // pass 1: sizes (parallel), prefix sum; pass 2: write
  std::vector<uint32_t> sz(count);
  parallel(count, threads, [&](uint64_t a, uint64_t b) {
    for (uint64_t k = a; k < b; ++k) sz[k] = static_cast<uint32_t>(gen_one(start + k, nullptr));
  });
  uint64_t total = 0;
  for (uint64_t k = 0; k < count; ++k) total += sz[k];
  if (!arena) return total;
  if (total > cap) return 0;
  uint64_t o = 0;
  for (uint64_t k = 0; k < count; ++k) {
    offsets[k] = o;
    o += sz[k];
  }
  parallel(count, threads, [&](uint64_t a, uint64_t b) {
    for (uint64_t k = a; k < b; ++k) gen_one(start + k, arena + offsets[k]);
  });
  return total;
}

// Bytes of records [start, start + count) summed per block of `block`
// records (sizes only, nothing written): the input of byte-balanced shard
// bounds over a batch too large to generate on one rank (cilium_amd/dist.py).
void l7g_block_bytes(int config, uint64_t seed, uint32_t n_rules, uint64_t start, uint64_t count, uint64_t block,
                     uint64_t* out, int threads) {
  const uint64_t nb = (count + block - 1) / block;
  parallel(nb, threads, [&](uint64_t a, uint64_t b) {
    for (uint64_t j = a; j < b; ++j) {
      const uint64_t lo = start + j * block, n = std::min(block, count - j * block);
      out[j] = l7g_requests(config, seed, n_rules, lo, n, nullptr, 0, nullptr, 1);
    }
  });
}

}  // extern "C"
