// l7m_internal.h — host-side pieces shared by the compilers and the C ABI.
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/l7match.h"
#include "program.h"

namespace l7m {

// program.h name hash of a host string (Kafka topic / ClientID tables, HTTP
// header-name table).
inline uint32_t name_hash(const std::string& s) {
  const size_t words = (s.size() + 3) / 4;
  uint32_t h = 0;
  for (size_t k = 0; k < words; ++k) {
    uint32_t w = 0;
    for (size_t b = 0; b < 4; ++b)
      if (4 * k + b < s.size()) w |= static_cast<uint32_t>(static_cast<unsigned char>(s[4 * k + b])) << (8 * b);
    h = name_hash_step(h, w);
  }
  return name_hash_final(h, static_cast<uint32_t>(s.size()));
}

constexpr uint32_t kDefaultLdsBudget = 48u * 1024u;  // bytes of DFA tables in the LDS image
constexpr uint32_t kLdsCtBudget = 24u * 1024u;       // ... including candidate tables

// One getHTTPRule HeaderMatcher (pkg/envoy/server.go:261-320).
struct HeaderMatcher {
  std::string name;   // as emitted by getHTTPRule (not lower-cased)
  std::string value;
  bool has_regex = false;  // HeaderMatcher.Regex != nil
  bool regex = false;      // Regex.Value
};

// Envoy HeaderData kind after construction (Regex / Value / Present).
enum class MatchKind : uint32_t { Regex = 0, Value = 1, Present = 2 };

struct CompileResult {
  int status = L7M_OK;
  std::string err;
  std::vector<uint32_t> program;
  l7m_ruleset_info info{};
  std::vector<std::string> names;         // HTTP: endpoint policy names (index = record policy)
  std::vector<l7m_rule_origin> origin;    // HTTP: per verdict index
};

// The port-entry structure of a compiled HTTP map (NetworkPolicyMap ->
// PolicyInstance -> PortNetworkPolicy, envoy/cilium_network_policy.h:40-208).
struct PolicyPlan {
  bool single = true;                      // one entry for every policy-0 key (l7m_compile_http)
  uint32_t n_policies = 1;
  std::vector<uint32_t> rule_entry;        // per flattened rule
  std::vector<std::pair<uint32_t, uint32_t>> keys;  // ent_key -> entry
  std::vector<uint8_t> entry_have_http;    // PortNetworkPolicyRules::have_http_rules_
  std::vector<std::string> names;
  std::vector<l7m_rule_origin> origin;
};

int translate_http_rule(const l7m_http_rule& r, std::vector<HeaderMatcher>* out, std::string* err);
MatchKind envoy_kind(const HeaderMatcher& m);
std::string lower_ascii(const std::string& s);

CompileResult compile_http(const l7m_http_rule* rules, size_t n, const l7m_opts& opts);
CompileResult compile_http_policies(const l7m_network_policy* pols, size_t n, const l7m_opts& opts);
CompileResult compile_kafka(const l7m_kafka_rule* rules, size_t n, const l7m_opts& opts);
CompileResult compile_kafka_map(const l7m_kafka_selector_rules* map, size_t n_entries,
                                const l7m_identity_selectors* ids, size_t n_ids, const l7m_opts& opts);

}  // namespace l7m

// The opaque handle.  Immutable after compile except for the per-device
// program copies, which are created lazily under `mu`.
inline uint64_t next_ruleset_serial() {
  static std::atomic<uint64_t> n{0};
  return ++n;
}

struct l7m_ruleset {
  std::atomic<int> refs{1};
  uint64_t serial = next_ruleset_serial();  // unique per handle (resident evaluator image cache key)
  uint32_t proto = 0;
  std::vector<uint32_t> program;
  l7m_ruleset_info info{};
  std::vector<std::string> names;       // HTTP endpoint policy names
  std::vector<l7m_rule_origin> origin;  // HTTP verdict index -> NPDS position
  std::mutex mu;
  void* dprog[64] = {nullptr};  // per HIP device
};
