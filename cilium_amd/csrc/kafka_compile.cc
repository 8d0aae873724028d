// kafka_compile.cc — compile []PortRuleKafka into the Kafka device program.
//
// Cold path, once per policy revision.  Restates PortRuleKafka.Sanitize
// (pkg/policy/api/rule_validation.go:190-233) with MapRoleToAPIKey
// (pkg/policy/api/kafka.go:274-293) and KafkaAPIKeyMap (kafka.go:153-188),
// then lays out what the device evaluator (l7m_kafka.hip) needs to compute
// (*RequestMessage).MatchesRule (pkg/kafka/policy.go:200-225) with a
// deterministic deciding-rule index:
//   * per request kind k (0..63; 64 = any other value) the ascending ids of
//     the rules whose CheckAPIKeyRole(k) holds (kafka.go:248-261): all of
//     them, and those with Topic == "";
//   * an open-addressed table Topic -> ascending ids of the rules with that
//     Topic (the reqTopicsMap coverage walk of policy.go:210-223);
//   * per rule: apiKeyInt mask, apiVersionInt, interned ClientID; a table
//     ClientID -> index resolves a request's ClientID once.
#include <algorithm>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "l7m_internal.h"
#include "program.h"

namespace l7m {
namespace {

std::string cstr(const char* p) { return p ? std::string(p) : std::string(); }

// KafkaAPIKeyMap (pkg/policy/api/kafka.go:153-188); index = apiKey value.
const char* const kApiKeyNames[] = {
    "produce", "fetch", "offsets", "metadata", "leaderandisr", "stopreplica",
    "updatemetadata", "controlledshutdown", "offsetcommit", "offsetfetch", "findcoordinator",
    "joingroup", "heartbeat", "leavegroup", "syncgroup", "describegroups", "listgroups",
    "saslhandshake", "apiversions", "createtopics", "deletetopics", "deleterecords",
    "initproducerid", "offsetforleaderepoch", "addpartitionstotxn", "addoffsetstotxn", "endtxn",
    "writetxnmarkers", "txnoffsetcommit", "describeacls", "createacls", "deleteacls",
    "describeconfigs", "alterconfigs"};

// Go strings.ToLower as far as it can decide equality with an ASCII name:
// ASCII upper case plus the two non-ASCII runes whose Unicode simple
// lower-case mapping is ASCII (U+0130 -> 'i', U+212A KELVIN SIGN -> 'k').
// Every other non-ASCII rune maps to a non-ASCII rune and cannot match.
std::string go_lower_ascii_names(const std::string& s) {
  std::string r;
  for (size_t i = 0; i < s.size();) {
    unsigned char c = static_cast<unsigned char>(s[i]);
    if (c == 0xC4 && i + 1 < s.size() && static_cast<unsigned char>(s[i + 1]) == 0xB0) {
      r += 'i';
      i += 2;
    } else if (c == 0xE2 && i + 2 < s.size() && static_cast<unsigned char>(s[i + 1]) == 0x84 &&
               static_cast<unsigned char>(s[i + 2]) == 0xAA) {
      r += 'k';
      i += 3;
    } else {
      r += (c >= 'A' && c <= 'Z') ? static_cast<char>(c - 'A' + 'a') : static_cast<char>(c);
      ++i;
    }
  }
  return r;
}

// strconv.ParseInt(s, 10, 16): optional sign, decimal digits, int16 range.
bool go_parse_int16(const std::string& s, int16_t* out) {
  size_t i = 0;
  bool neg = false;
  if (!s.empty() && (s[0] == '+' || s[0] == '-')) {
    neg = s[0] == '-';
    i = 1;
  }
  if (i >= s.size()) return false;
  int64_t v = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
    if (v > 100000) v = 100000;  // saturate: already out of range
  }
  if (neg) v = -v;
  if (v < -32768 || v > 32767) return false;
  *out = static_cast<int16_t>(v);
  return true;
}

// KafkaTopicValidChar `^[a-zA-Z0-9\\._\\-]+$` (kafka.go:244); in the Go raw
// string the class also admits a backslash.
bool topic_chars_valid(const std::string& t) {
  if (t.empty()) return false;
  for (unsigned char c : t) {
    bool ok = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') ||
              c == '\\' || c == '.' || c == '_' || c == '-';
    if (!ok) return false;
  }
  return true;
}

struct KRule {
  std::vector<int> keys;  // apiKeyInt (empty = any kind)
  bool has_version = false;
  int16_t version = 0;
  std::string client, topic;
};

// PortRuleKafka.Sanitize (rule_validation.go:190-233).
int sanitize(const l7m_kafka_rule& in, KRule* r, std::string* err) {
  const std::string role = cstr(in.role), key = cstr(in.api_key), ver = cstr(in.api_version);
  r->client = cstr(in.client_id);
  r->topic = cstr(in.topic);
  if (!key.empty() && !role.empty()) {
    *err = "Cannot set both Role:\"" + role + "\" and APIKey :\"" + key + "\" together";
    return L7M_EINVAL_RULE;
  }
  if (!key.empty()) {
    const std::string lk = go_lower_ascii_names(key);
    int found = -1;
    for (int k = 0; k < static_cast<int>(sizeof(kApiKeyNames) / sizeof(*kApiKeyNames)); ++k)
      if (lk == kApiKeyNames[k]) found = k;
    if (found < 0) {
      *err = "invalid Kafka APIKey :\"" + key + "\"";
      return L7M_EINVAL_RULE;
    }
    r->keys.push_back(found);
  }
  if (!role.empty()) {  // MapRoleToAPIKey (kafka.go:274-293)
    const std::string lr = go_lower_ascii_names(role);
    if (lr == "produce") {
      r->keys = {0, 3, 18};
    } else if (lr == "consume") {
      r->keys = {1, 2, 3, 8, 9, 10, 11, 12, 13, 14, 18};
    } else {
      *err = "invalid Kafka APIRole :\"" + role + "\"";
      return L7M_EINVAL_RULE;
    }
  }
  if (!ver.empty()) {
    if (!go_parse_int16(ver, &r->version)) {
      *err = "invalid Kafka APIVersion :\"" + ver + "\"";
      return L7M_EINVAL_RULE;
    }
    r->has_version = true;
  }
  if (!r->topic.empty()) {
    if (r->topic.size() > 255) {
      *err = "kafka topic exceeds maximum len of 255";
      return L7M_EINVAL_RULE;
    }
    if (!topic_chars_valid(r->topic)) {
      *err = "invalid Kafka Topic name \"" + r->topic + "\"";
      return L7M_EINVAL_RULE;
    }
  }
  return L7M_OK;
}


bool key_ok(const KRule& r, uint32_t k) {  // CheckAPIKeyRole for table index k
  if (r.keys.empty()) return true;
  if (k >= 64) return false;
  for (int x : r.keys)
    if (static_cast<uint32_t>(x) == k) return true;
  return false;
}

}  // namespace

CompileResult compile_kafka(const l7m_kafka_rule* rules, size_t n, const l7m_opts& opts) {
  const l7m_kafka_selector_rules all{rules, n, 1u, 0u};
  return compile_kafka_map(&all, 1, nullptr, 0, opts);
}

// The rules of every L7DataMap entry, flattened entry by entry (verdict index
// order); rule i applies to a source whose selector mask has bit group[i].
CompileResult compile_kafka_map(const l7m_kafka_selector_rules* map, size_t n_entries,
                                const l7m_identity_selectors* ids, size_t n_ids, const l7m_opts& opts) {
  (void)opts;
  CompileResult res;
  auto fail = [&](int st, const std::string& m) {
    res.status = st;
    res.err = m;
    return res;
  };
  if (n_entries > 0 && !map) return fail(L7M_EINVAL, "map == NULL");
  if (n_ids > 0 && !ids) return fail(L7M_EINVAL, "identities == NULL");
  if (n_entries > kMaxKafkaGroups)
    return fail(L7M_ETOOBIG, std::to_string(n_entries) + " L7DataMap entries > " + std::to_string(kMaxKafkaGroups));
  uint64_t wild = 0;
  bool selective = false;
  size_t n = 0;
  for (size_t g = 0; g < n_entries; ++g) {
    if (map[g].n_rules > 0 && !map[g].rules) return fail(L7M_EINVAL, "entry " + std::to_string(g) + ": rules == NULL");
    n += map[g].n_rules;
    if (map[g].wildcard) wild |= 1ull << g;
    else selective = true;
  }
  if (n >= (1u << 30)) return fail(L7M_ETOOBIG, "too many rules");

  std::vector<KRule> kr(n);
  std::vector<uint32_t> group(n);
  for (size_t g = 0, i = 0; g < n_entries; ++g)
    for (size_t j = 0; j < map[g].n_rules; ++j, ++i) {
      std::string err;
      int rc = sanitize(map[g].rules[j], &kr[i], &err);
      if (rc != L7M_OK) return fail(rc, "rule " + std::to_string(i) + ": " + err);
      group[i] = static_cast<uint32_t>(g);
    }

  // string area: client ids and distinct topics
  std::string strings;
  auto put_str = [&](const std::string& s) {
    uint32_t o = static_cast<uint32_t>(strings.size());
    strings += s;
    return o;
  };
  std::vector<KafkaRuleDesc> desc(n);
  std::map<std::string, std::vector<uint32_t>> by_topic;
  std::map<std::string, uint32_t> client_ids;
  for (size_t i = 0; i < n; ++i) {
    const KRule& r = kr[i];
    KafkaRuleDesc& d = desc[i];
    std::memset(&d, 0, sizeof d);
    d.client_idx = kNone;
    d.group = group[i];
    if (r.keys.empty()) d.flags |= kKRuleAnyKey;
    for (int k : r.keys) {
      if (k < 32) d.keys_lo |= 1u << k;
      else d.keys_hi |= 1u << (k - 32);
    }
    if (r.has_version) {
      d.flags |= kKRuleVersion;
      d.version = r.version;
    }
    if (!r.client.empty()) {
      d.flags |= kKRuleClient;
      auto it = client_ids.emplace(r.client, static_cast<uint32_t>(client_ids.size())).first;
      d.client_idx = it->second;
    }
    if (!r.topic.empty()) {
      d.flags |= kKRuleTopic;
      by_topic[r.topic].push_back(static_cast<uint32_t>(i));
    }
  }

  std::vector<uint32_t> pool;
  auto push_list = [&](const std::vector<uint32_t>& v) -> Span {
    Span s{static_cast<uint32_t>(pool.size()), static_cast<uint32_t>(v.size())};
    pool.insert(pool.end(), v.begin(), v.end());
    return s;
  };

  KafkaHeader h;
  std::memset(&h, 0, sizeof h);
  h.magic = kMagicKafka;
  h.n_rules = static_cast<uint32_t>(n);
  for (uint32_t k = 0; k < kKafkaKinds; ++k) {
    std::vector<uint32_t> all, notopic;
    for (size_t i = 0; i < n; ++i)
      if (key_ok(kr[i], k)) {
        all.push_back(static_cast<uint32_t>(i));
        if (kr[i].topic.empty()) notopic.push_back(static_cast<uint32_t>(i));
      }
    h.all_by_kind[k] = push_list(all);
    h.notopic_by_kind[k] = push_list(notopic);
  }

  auto table_size = [](size_t keys) -> uint32_t {  // load factor <= 1/2
    if (!keys) return 0;
    uint32_t m = 2;
    while (m < 2 * keys) m <<= 1;
    return m;
  };
  auto put_prefix = [](uint32_t* pfx, size_t cap, const std::string& s) {
    std::memcpy(pfx, s.data(), std::min(cap, s.size()));
  };
  // Distinct apiKey sets; id 0 = any kind.
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> kset_ids;
  std::vector<uint64_t> kset_masks(1, ~0ull);
  auto kset_of = [&](const KafkaRuleDesc& d) -> uint32_t {
    if (d.flags & kKRuleAnyKey) return 0;
    auto it = kset_ids.emplace(std::make_pair(d.keys_lo, d.keys_hi), static_cast<uint32_t>(kset_masks.size()));
    if (it.second) kset_masks.push_back((static_cast<uint64_t>(d.keys_hi) << 32) | d.keys_lo);
    return it.first->second;
  };
  const uint32_t n_slots = table_size(by_topic.size());
  std::vector<KafkaTopicSlot> slots(n_slots);
  std::vector<KafkaTopicExt> ext(n_slots);
  std::memset(slots.data(), 0, slots.size() * sizeof(KafkaTopicSlot));
  std::memset(ext.data(), 0, ext.size() * sizeof(KafkaTopicExt));
  for (const auto& kv : by_topic) {
    const uint32_t hk = name_hash(kv.first);
    uint32_t at = hk & (n_slots - 1);
    while (slots[at].hash != 0) at = (at + 1) & (n_slots - 1);
    KafkaTopicSlot& sl = slots[at];
    const KafkaRuleDesc& d = desc[kv.second[0]];
    sl.hash = hk;
    sl.meta = static_cast<uint32_t>(kv.first.size()) | (kset_of(d) << 8) |
              ((d.flags & kKRuleVersion) ? kSlotVersionCond : 0u) | ((d.flags & kKRuleClient) ? kSlotClientCond : 0u) |
              (static_cast<uint32_t>(static_cast<uint16_t>(d.version)) << 16);
    sl.r0 = kv.second[0] | (kv.second.size() > 1 ? kSlotMore : 0u);
    sl.r0_client = (d.client_idx == kNone ? 0xffffu : d.client_idx) | (d.group << 16);
    put_prefix(sl.pfx, kTopicInline, kv.first);
    ext[at].str_off = put_str(kv.first);
    ext[at].rules = push_list(kv.second);
  }
  if (kset_masks.size() > kMaxKsets) return fail(L7M_ETOOBIG, "too many distinct apiKey sets");
  uint64_t kind_ok[kKafkaKinds];
  for (uint32_t k = 0; k < kKafkaKinds; ++k) {
    kind_ok[k] = 1;  // kset 0: any kind
    for (uint32_t s = 1; s < kset_masks.size(); ++s)
      if (k < 64 && ((kset_masks[s] >> k) & 1)) kind_ok[k] |= 1ull << s;
  }

  if (client_ids.size() >= 0xffffu) return fail(L7M_ETOOBIG, "more than 65534 distinct ClientIDs");
  const uint32_t n_clients = table_size(client_ids.size());
  std::vector<KafkaClientSlot> cslots(n_clients);
  std::memset(cslots.data(), 0, cslots.size() * sizeof(KafkaClientSlot));
  for (const auto& kv : client_ids) {
    uint32_t hk = name_hash(kv.first);
    uint32_t at = hk & (n_clients - 1);
    while (cslots[at].hash != 0) at = (at + 1) & (n_clients - 1);
    KafkaClientSlot& sl = cslots[at];
    sl.hash = hk;
    sl.str_off = put_str(kv.first);
    sl.str_len = static_cast<uint32_t>(kv.first.size());
    sl.idx = kv.second;
    put_prefix(sl.pfx, kClientInline, kv.first);
  }

  // source identity -> selector mask (only when some entry is not the wildcard)
  const uint32_t n_id_slots = selective ? std::max<uint32_t>(2, table_size(n_ids)) : 0;
  std::vector<KafkaIdSlot> id_slots(1 + n_id_slots);
  std::memset(id_slots.data(), 0, id_slots.size() * sizeof(KafkaIdSlot));
  id_slots[0].mask_lo = static_cast<uint32_t>(wild);
  id_slots[0].mask_hi = static_cast<uint32_t>(wild >> 32);
  for (size_t k = 0; k < n_ids && n_id_slots; ++k) {
    const l7m_identity_selectors& e = ids[k];
    if (e.identity == 0) return fail(L7M_EINVAL, "identity 0 is the unresolved source (no selector matches it)");
    if (e.n_selectors > 0 && !e.selectors) return fail(L7M_EINVAL, "identity " + std::to_string(e.identity) +
                                                                       ": selectors == NULL");
    uint64_t m = wild;
    for (size_t j = 0; j < e.n_selectors; ++j) {
      if (e.selectors[j] >= n_entries)
        return fail(L7M_EINVAL, "identity " + std::to_string(e.identity) + ": selector " +
                                    std::to_string(e.selectors[j]) + " out of range");
      m |= 1ull << e.selectors[j];
    }
    uint32_t at = kafka_id_hash(e.identity) & (n_id_slots - 1);
    while (id_slots[1 + at].identity != 0) {
      if (id_slots[1 + at].identity == e.identity)
        return fail(L7M_EINVAL, "identity " + std::to_string(e.identity) + " listed twice");
      at = (at + 1) & (n_id_slots - 1);
    }
    id_slots[1 + at].identity = e.identity;
    id_slots[1 + at].mask_lo = static_cast<uint32_t>(m);
    id_slots[1 + at].mask_hi = static_cast<uint32_t>(m >> 32);
  }

  uint32_t crc[256];
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    crc[i] = c;
  }

  uint64_t w = sizeof(KafkaHeader) / 4;
  auto take = [&](uint64_t words) {  // 16-byte aligned sections
    w = (w + 3) & ~uint64_t(3);
    uint64_t o = w;
    w += words;
    return static_cast<uint32_t>(o);
  };
  h.off_rules = take(static_cast<uint64_t>(n) * sizeof(KafkaRuleDesc) / 4);
  h.off_slots = take(static_cast<uint64_t>(n_slots) * sizeof(KafkaTopicSlot) / 4);
  h.n_slots = n_slots;
  h.off_ext = take(static_cast<uint64_t>(n_slots) * sizeof(KafkaTopicExt) / 4);
  h.off_kind_ok = take(2 * kKafkaKinds);
  h.off_clients = take(static_cast<uint64_t>(n_clients) * sizeof(KafkaClientSlot) / 4);
  h.n_clients = n_clients;
  h.off_pool = take(pool.size());
  h.off_crc = take(256);
  h.off_strings = take((strings.size() + 3) / 4);
  h.off_ids = take(static_cast<uint64_t>(1 + n_id_slots) * sizeof(KafkaIdSlot) / 4);
  h.n_id_slots = n_id_slots;
  if (w >= (1ull << 32)) return fail(L7M_ETOOBIG, "program exceeds 16 GiB");
  h.total_words = static_cast<uint32_t>(w);

  std::vector<uint32_t> prog(w, 0);
  std::memcpy(prog.data(), &h, sizeof h);
  if (n) std::memcpy(prog.data() + h.off_rules, desc.data(), n * sizeof(KafkaRuleDesc));
  if (n_slots) std::memcpy(prog.data() + h.off_slots, slots.data(), n_slots * sizeof(KafkaTopicSlot));
  if (n_slots) std::memcpy(prog.data() + h.off_ext, ext.data(), n_slots * sizeof(KafkaTopicExt));
  std::memcpy(prog.data() + h.off_kind_ok, kind_ok, sizeof kind_ok);
  if (n_clients)
    std::memcpy(prog.data() + h.off_clients, cslots.data(), n_clients * sizeof(KafkaClientSlot));
  if (!pool.empty()) std::memcpy(prog.data() + h.off_pool, pool.data(), pool.size() * 4);
  std::memcpy(prog.data() + h.off_crc, crc, sizeof crc);
  if (!strings.empty()) std::memcpy(prog.data() + h.off_strings, strings.data(), strings.size());
  std::memcpy(prog.data() + h.off_ids, id_slots.data(), id_slots.size() * sizeof(KafkaIdSlot));

  res.program = std::move(prog);
  res.info.proto = L7M_PROTO_KAFKA;
  res.info.n_rules = static_cast<uint32_t>(n);
  res.info.program_bytes = w * 4;
  res.info.n_counters = static_cast<uint32_t>(n) + 2;
  return res;
}

}  // namespace l7m
