"""Writes tests/golden/*.json: known-answer vectors TRANSCRIBED from the
reference's own tests and docs (data only: inputs and expected outputs).

Sources (paths relative to the uniberg/cilium tree):
  envoy/cilium_integration_test.cc:40-75   BASIC_POLICY (NPDS, ingress+egress port 80)
  envoy/cilium_integration_test.cc:89-93   test identity: remote_id 1, port 80
  envoy/cilium_integration_test.cc:605-639 ingress Accepted/Denied cases
  envoy/cilium_integration_test.cc:683-717 egress cases (same expectations)
  pkg/envoy/envoy/api/v2/route/route.pb.go:2426-2430  \\d{3} doc examples
  pkg/envoy/server_test.go:40-107,334-337  getHTTPRule translation (ExpectedHeaders1..3)
  README.rst:36-41 + SURVEY.md §0.4         README policy semantics (literal header value)
  pkg/kafka/policy_test.go:61-127           MatchesRule topic coverage / unknown kinds
  pkg/proxy/kafka_test.go:184-258           proxy allow/deny by topic
  examples/policies/l7/{http,kafka}/*.json  rule-import fixtures

The BASIC_POLICY NPDS rules are already in Envoy form (header matchers); they
are expressed here as the PortRuleHTTP values getHTTPRule maps onto exactly
those matchers (a ':path' literal is the header spec ":path <value>").
Run:  python tests/golden/make_golden.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

# --- envoy/cilium_integration_test.cc:40-75 ------------------------------
# remote_policies [1]: five http_rules; remote_policies [2]: one.
BASIC_POLICY_RULES = [
    {"Headers": [":path /allowed"], "RemoteIDs": [1]},
    {"Path": ".*public$", "RemoteIDs": [1]},
    {"Headers": [":authority allowedHOST"], "RemoteIDs": [1]},
    {"Host": ".*REGEX.*", "RemoteIDs": [1]},
    {"Headers": [":method PUT", ":path /public/opinions"], "RemoteIDs": [1]},
    {"Headers": [":path /only-2-allowed"], "RemoteIDs": [2]},
]
# identity 1 (cilium_integration_test.cc:89-93); expectations :605-639 / :683-717
BASIC_CASES = [
    ("DeniedPathPrefix", "GET", "/prefix", "host", False),
    ("AllowedPathPrefix", "GET", "/allowed", "host", True),
    ("AllowedPathRegex", "GET", "/maybe/public", "host", True),
    ("DeniedPath", "GET", "/maybe/private", "host", False),
    ("AllowedHostString", "GET", "/maybe/private", "allowedHOST", True),
    ("AllowedHostRegex", "GET", "/maybe/private", "hostREGEXname", True),
    ("DeniedMethod", "POST", "/maybe/private", "host", False),
    ("AcceptedMethod", "PUT", "/public/opinions", "host", True),
    ("L3DeniedPath", "GET", "/only-2-allowed", "host", False),
]

# route.pb.go:2426-2430
REGEX_DOC = [
    {"regex": "\\d{3}", "value": "123", "match": True},
    {"regex": "\\d{3}", "value": "1234", "match": False},
    {"regex": "\\d{3}", "value": "123.456", "match": False},
]

# server_test.go:40-107 (getHTTPRule) — Regex null = nil BoolValue
TRANSLATION = [
    {"rule": {"Path": "/foo", "Method": "GET", "Host": "foo.cilium.io",
              "Headers": ["header2 value", "header1"]},
     "expected": [{"Name": ":authority", "Value": "foo.cilium.io", "Regex": True},
                  {"Name": ":method", "Value": "GET", "Regex": True},
                  {"Name": ":path", "Value": "/foo", "Regex": True},
                  {"Name": "header1", "Value": "", "Regex": None},
                  {"Name": "header2", "Value": "value", "Regex": None}]},
    {"rule": {"Path": "/bar", "Method": "PUT"},
     "expected": [{"Name": ":method", "Value": "PUT", "Regex": True},
                  {"Name": ":path", "Value": "/bar", "Regex": True}]},
    {"rule": {"Path": "/bar", "Method": "GET"},
     "expected": [{"Name": ":method", "Value": "GET", "Regex": True},
                  {"Name": ":path", "Value": "/bar", "Regex": True}]},
]

# README.rst:36-41 policy; header value is a LITERAL (pkg/envoy/server.go:296-306)
README_RULES = [{"Method": "GET", "Path": "/public/.*", "Headers": ["X-Token: [0-9]+"]}]
README_CASES = [
    {"req": {"method": "GET", "path": "/public/a", "headers": [["x-token", "[0-9]+"]]}, "verdict": 0},
    {"req": {"method": "GET", "path": "/public/a", "headers": [["x-token", "123"]]}, "verdict": -1},
    {"req": {"method": "GET", "path": "/public/", "headers": [["x-token", "[0-9]+"]]}, "verdict": 0},
    {"req": {"method": "GET", "path": "/public", "headers": [["x-token", "[0-9]+"]]}, "verdict": -1},
    {"req": {"method": "POST", "path": "/public/a", "headers": [["x-token", "[0-9]+"]]}, "verdict": -1},
    {"req": {"method": "GET", "path": "/public/a", "headers": []}, "verdict": -1},
    {"req": {"method": "GET", "path": "/private/a", "headers": [["x-token", "[0-9]+"]]}, "verdict": -1},
    {"req": {"method": "GET", "path": "/public/a\n", "headers": [["x-token", "[0-9]+"]]}, "verdict": -1},
]

# examples/policies/l7/http/http.json
EXAMPLE_HTTP_RULES = [{"Method": "GET", "Path": "/path1$"},
                      {"Method": "PUT", "Path": "/path2$", "Headers": ["X-My-Header: true"]}]
EXAMPLE_HTTP_CASES = [
    {"req": {"method": "GET", "path": "/path1", "headers": []}, "verdict": 0},
    {"req": {"method": "GET", "path": "/path1/x", "headers": []}, "verdict": -1},
    {"req": {"method": "PUT", "path": "/path2", "headers": [["x-my-header", "true"]]}, "verdict": 1},
    {"req": {"method": "PUT", "path": "/path2", "headers": [["x-my-header", "false"]]}, "verdict": -1},
    {"req": {"method": "PUT", "path": "/path2", "headers": []}, "verdict": -1},
    {"req": {"method": "GET", "path": "/path2", "headers": [["x-my-header", "true"]]}, "verdict": -1},
]

# pkg/kafka/policy_test.go:61-108: produce request, topics foo+bar, kind 0 v0,
# client "test"; rules are unsanitized (apiKeyInt empty = any kind).
KAFKA_PRODUCE_FOO_BAR = {"kind": 0, "version": 0, "client": "test", "topics": ["foo", "bar"]}
KAFKA_POLICY_TEST = [
    {"rules": [], "allow": False},
    {"rules": [{}], "allow": True, "verdict": 0},
    {"rules": [{"Topic": "foo"}], "allow": False},
    {"rules": [{"Topic": "foo"}, {"Topic": "bar"}], "allow": True, "verdict": 1},
    {"rules": [{"Topic": "foo"}, {"Topic": "baz"}], "allow": False},
    {"rules": [{"Topic": "baz"}, {"Topic": "foo2"}], "allow": False},
    {"rules": [{"Topic": "bar"}, {"Topic": "foo"}], "allow": True, "verdict": 1},
    {"rules": [{"Topic": "bar"}, {"Topic": "foo"}, {"Topic": "baz"}], "allow": True, "verdict": 1},
]
# policy_test.go:112-127: unknown-kind whitelisting (kind 18 allowed, 19 not)
KAFKA_UNKNOWN = [
    {"kind": 18, "rules": [{"APIKey": "metadata"}, {"APIKey": "apiversions"}], "allow": True, "verdict": 1},
    {"kind": 19, "rules": [{"APIKey": "metadata"}, {"APIKey": "apiversions"}], "allow": False},
    {"kind": 18, "rules": [], "allow": False},
]
# kafka_test.go:184-258
KAFKA_PROXY_RULES = [{"APIKey": "metadata", "APIVersion": "0"},
                     {"APIKey": "produce", "APIVersion": "0", "Topic": "allowedTopic"}]
KAFKA_PROXY_CASES = [
    {"req": {"kind": 0, "version": 0, "client": "", "topics": ["allowedTopic"]}, "allow": True, "verdict": 1},
    {"req": {"kind": 0, "version": 0, "client": "", "topics": ["disallowedTopic"]}, "allow": False},
    {"req": {"kind": 3, "version": 0, "client": "", "topics": []}, "allow": True, "verdict": 0},
]
# examples/policies/l7/kafka/kafka.json, kafka-role.json
KAFKA_EXAMPLE_RULES = [{"APIKey": "apiversions"}, {"APIKey": "metadata"},
                       {"APIKey": "produce", "Topic": "deathstar-plans"},
                       {"APIKey": "produce", "Topic": "empire-announce"}]
KAFKA_ROLE_RULES = [{"Role": "produce", "Topic": "deathstar-plans"},
                    {"Role": "produce", "Topic": "empire-announce"}]
# Sanitize known answers (rule_validation.go:190-233)
KAFKA_SANITIZE = [
    {"rule": {"APIKey": "produce", "Role": "produce"}, "ok": False},
    {"rule": {"APIKey": "nosuchkey"}, "ok": False},
    {"rule": {"APIKey": "PRODUCE"}, "ok": True},
    {"rule": {"Role": "Consume"}, "ok": True},
    {"rule": {"Role": "admin"}, "ok": False},
    {"rule": {"APIVersion": "abc"}, "ok": False},
    {"rule": {"APIVersion": "32768"}, "ok": False},
    {"rule": {"APIVersion": "-1"}, "ok": True},
    {"rule": {"APIVersion": "+7"}, "ok": True},
    {"rule": {"Topic": "a" * 256}, "ok": False},
    {"rule": {"Topic": "a" * 255}, "ok": True},
    {"rule": {"Topic": "bad topic"}, "ok": False},
    {"rule": {"Topic": "ok.topic_name-1\\x"}, "ok": True},
]


# The same BASIC_POLICY as the NPDS resource it is (name '173', ingress and
# egress port 80, two PortNetworkPolicyRules), with the directions of the
# ingress (:605-639, remote identity 1) and egress (:683-717, destination
# resolved to identity 1 by the host map :670-678) tests, and the
# DuplicatePort test (:641-659): the policy is rejected, so the endpoint has
# no policy and every request is denied (403).
_BASIC_PORT = {"Port": 80, "Rules": [
    {"RemotePolicies": [1], "HttpRules": [r for r in BASIC_POLICY_RULES if r["RemoteIDs"] == [1]]},
    {"RemotePolicies": [2], "HttpRules": [r for r in BASIC_POLICY_RULES if r["RemoteIDs"] == [2]]},
]}
for _r in _BASIC_PORT["Rules"]:
    _r["HttpRules"] = [{k: v for k, v in h.items() if k != "RemoteIDs"} for h in _r["HttpRules"]]
NPDS_BASIC = {"Name": "173", "Ingress": [_BASIC_PORT], "Egress": [_BASIC_PORT]}
NPDS_DUPLICATE_PORT = {"Name": "173", "Ingress": [_BASIC_PORT, {"Port": 80, "Rules": [
    {"RemotePolicies": [2], "HttpRules": [{"Headers": [":path /only-2-allowed"]}]}]}], "Egress": [_BASIC_PORT]}


def main():
    out = {
        "npds_basic_policy": {"source": "envoy/cilium_integration_test.cc:40-75,89-100,605-717",
                              "policy": NPDS_BASIC, "remote_id": 1, "dport": 80,
                              "ingress_cases": [{"name": n, "method": m, "path": p, "authority": a, "allow": ok}
                                                for n, m, p, a, ok in BASIC_CASES],
                              "egress_cases": [{"name": n, "method": m, "path": p, "authority": a, "allow": ok}
                                               for n, m, p, a, ok in BASIC_CASES],
                              "duplicate_port_policy": NPDS_DUPLICATE_PORT,
                              "duplicate_port_case": {"name": "DuplicatePort", "method": "GET", "path": "/allowed",
                                                      "authority": "host", "allow": False}},
        "basic_policy": {"source": "envoy/cilium_integration_test.cc:40-75,605-639,683-717",
                         "rules": BASIC_POLICY_RULES, "remote_id": 1, "dport": 80,
                         "cases": [{"name": n, "method": m, "path": p, "authority": a, "allow": ok}
                                   for n, m, p, a, ok in BASIC_CASES]},
        "regex_doc": {"source": "pkg/envoy/envoy/api/v2/route/route.pb.go:2426-2430", "cases": REGEX_DOC},
        "translation": {"source": "pkg/envoy/server_test.go:40-107", "cases": TRANSLATION},
        "readme": {"source": "README.rst:36-41; pkg/envoy/server.go:296-306", "rules": README_RULES,
                   "cases": README_CASES},
        "example_http": {"source": "examples/policies/l7/http/http.json", "rules": EXAMPLE_HTTP_RULES,
                         "cases": EXAMPLE_HTTP_CASES},
    }
    with open(os.path.join(HERE, "http_known_answers.json"), "w") as f:
        json.dump(out, f, indent=1)
    kout = {
        "policy_test": {"source": "pkg/kafka/policy_test.go:61-108", "request": KAFKA_PRODUCE_FOO_BAR,
                        "cases": KAFKA_POLICY_TEST},
        "unknown_kind": {"source": "pkg/kafka/policy_test.go:112-127", "cases": KAFKA_UNKNOWN},
        "proxy": {"source": "pkg/proxy/kafka_test.go:184-258", "rules": KAFKA_PROXY_RULES,
                  "cases": KAFKA_PROXY_CASES},
        "examples": {"source": "examples/policies/l7/kafka/kafka.json, kafka-role.json",
                     "rules": KAFKA_EXAMPLE_RULES, "role_rules": KAFKA_ROLE_RULES},
        "sanitize": {"source": "pkg/policy/api/rule_validation.go:190-233", "cases": KAFKA_SANITIZE},
    }
    with open(os.path.join(HERE, "kafka_known_answers.json"), "w") as f:
        json.dump(kout, f, indent=1)


if __name__ == "__main__":
    main()
