"""NPDS policy maps (NetworkPolicyMap::Allowed, envoy/cilium_network_policy.h
:40-237) on the CPU: the oracle pinned by the reference's integration-test
known answers (ingress AND egress, envoy/cilium_integration_test.cc:605-717,
DuplicatePort :641-659), and the compiled program (tests/program_interp.py)
against the oracle on random multi-policy, multi-port, two-direction maps."""
import numpy as np
import pytest

from cilium_amd import l7match as L
from oracle import OracleError, PolicyOracle
from policy_cases import basic_requests, golden_npds, npds, random_policies, random_requests
from program_interp import HttpProgram


def test_oracle_npds_known_answers_ingress_and_egress():
    g = golden_npds()
    pols = [npds(g["policy"])]
    reqs, expect = basic_requests(g)
    arena, offs = L.pack_http(reqs)
    v = PolicyOracle(pols).eval(arena, offs)
    assert [(x >= 0) for x in v.tolist()] == expect
    # the allowing index names an HTTP rule of the remote-1 port rule
    rs = L.RuleSet.compile_http_policies(pols)
    for x, q in zip(v.tolist(), reqs):
        if x >= 0:
            pol, ingress, port, port_rule, http_rule = rs.rule_origin(x)
            assert (pol, ingress, port, port_rule) == (0, q.ingress, 80, 0) and http_rule >= 0


def test_compiled_npds_known_answers_match_oracle():
    g = golden_npds()
    pols = [npds(g["policy"])]
    reqs, expect = basic_requests(g)
    arena, offs = L.pack_http(reqs)
    rs = L.RuleSet.compile_http_policies(pols)
    got = HttpProgram(rs.program()).eval(arena, offs)
    exp = PolicyOracle(pols).eval(arena, offs)
    assert got.tolist() == exp.tolist()
    assert [(x >= 0) for x in got.tolist()] == expect


def test_duplicate_port_is_rejected_and_endpoint_then_denies():
    """DuplicatePort (cilium_integration_test.cc:641-659): Envoy throws
    "Duplicate port number", the policy is not installed, the endpoint has
    no policy and its requests are denied."""
    g = golden_npds()
    bad = [npds(g["duplicate_port_policy"])]
    with pytest.raises(L.L7Error) as e:
        L.RuleSet.compile_http_policies(bad)
    assert e.value.code == L.L7M_EINVAL_RULE and "Duplicate port" in str(e.value)
    with pytest.raises(OracleError):
        PolicyOracle(bad)
    # the map without that endpoint: its name resolves to no policy -> deny
    rs = L.RuleSet.compile_http_policies([])
    assert rs.policy_index("173") == L.POLICY_UNKNOWN
    c = g["duplicate_port_case"]
    arena, offs = L.pack_http([L.HTTPRequest(c["method"], c["path"], c["authority"], remote_id=1, dport=80,
                                             policy=L.POLICY_UNKNOWN)])
    assert HttpProgram(rs.program()).eval(arena, offs).tolist() == [L.VERDICT_DENY]
    assert PolicyOracle([]).eval(arena, offs).tolist() == [L.VERDICT_DENY]


def test_policy_compile_errors():
    empty_http = L.NetworkPolicy("e", Ingress=[L.PortNetworkPolicy(80, [L.PortNetworkPolicyRule(HttpRules=[])])])
    with pytest.raises(L.L7Error) as e:
        L.RuleSet.compile_http_policies([empty_http])
    assert e.value.code == L.L7M_EINVAL_RULE  # HttpNetworkPolicyRules.http_rules min_items = 1
    with pytest.raises(L.L7Error) as e:
        L.RuleSet.compile_http_policies([L.NetworkPolicy("a"), L.NetworkPolicy("a")])
    assert e.value.code == L.L7M_EINVAL_RULE
    with pytest.raises(L.L7Error) as e:
        L.RuleSet.compile_http_policies([L.NetworkPolicy("p", Ingress=[L.PortNetworkPolicy(70000)])])
    assert e.value.code == L.L7M_EINVAL_RULE
    bad_re = L.NetworkPolicy("r", Egress=[L.PortNetworkPolicy(0, [L.PortNetworkPolicyRule(
        HttpRules=[L.PortRuleHTTP(Path="(")])])])
    with pytest.raises(L.L7Error) as e:
        L.RuleSet.compile_http_policies([bad_re])
    assert e.value.code == L.L7M_EINVAL_REGEX


def test_port_selection_semantics():
    """Exact port, then port 0, then no entry -> allow; entries without HTTP
    rules allow; UDP entries are not installed; unknown policy denies."""
    pol = L.NetworkPolicy("ep", Ingress=[
        L.PortNetworkPolicy(0, [L.PortNetworkPolicyRule(HttpRules=[L.PortRuleHTTP(Path="/zero")])]),
        L.PortNetworkPolicy(80, [L.PortNetworkPolicyRule(HttpRules=[L.PortRuleHTTP(Path="/eighty")])]),
        L.PortNetworkPolicy(81, []),                                          # no rules: allow all
        L.PortNetworkPolicy(82, [L.PortNetworkPolicyRule(RemotePolicies=[7])]),  # no HTTP rules: allow all
        L.PortNetworkPolicy(83, [L.PortNetworkPolicyRule(HttpRules=[L.PortRuleHTTP(Path="/u")])], Protocol=L.L4_UDP),
    ], Egress=[L.PortNetworkPolicy(80, [L.PortNetworkPolicyRule(HttpRules=[L.PortRuleHTTP(Path="/out")])])])
    rs = L.RuleSet.compile_http_policies([pol])
    assert rs.policy_index("ep") == 0
    cases = [  # (path, dport, ingress, policy, expected)
        ("/eighty", 80, True, 0, 0),          # exact port rule (index 0: port 80 entry first)
        ("/zero", 80, True, 0, 2),            # falls through to port 0 (indexed last)
        ("/nope", 80, True, 0, L.VERDICT_DENY),
        ("/zero", 9, True, 0, 2),             # no exact entry: port 0 decides
        ("/x", 81, True, 0, L.VERDICT_ALLOW_NO_L7),
        ("/x", 82, True, 0, L.VERDICT_ALLOW_NO_L7),
        ("/u", 83, True, 0, L.VERDICT_DENY),  # UDP entry absent: port 0 rules apply
        ("/out", 80, False, 0, 3),
        ("/out", 90, False, 0, L.VERDICT_ALLOW_NO_PORT_POLICY),
        ("/eighty", 80, True, L.POLICY_UNKNOWN, L.VERDICT_DENY),
        ("/eighty", 80, True, 1, L.VERDICT_DENY),
    ]
    reqs = [L.HTTPRequest("GET", p, "h", dport=d, ingress=i, policy=pp) for p, d, i, pp, _ in cases]
    arena, offs = L.pack_http(reqs)
    exp = [c[-1] for c in cases]
    assert PolicyOracle([pol]).eval(arena, offs).tolist() == exp
    assert HttpProgram(rs.program()).eval(arena, offs).tolist() == exp
    # index order: port 80 (0), port 82's matcher-less pseudo rule (1), port 0 (2), egress 80 (3)
    assert rs.rule_origin(1) == (0, True, 82, 0, -1)
    assert rs.rule_origin(2) == (0, True, 0, 0, 0)
    assert rs.rule_origin(3) == (0, False, 80, 0, 0)


def test_flat_rule_set_is_one_policy_for_every_port_and_direction():
    rs = L.RuleSet.compile_http([L.PortRuleHTTP(Path="/a")])
    reqs = [L.HTTPRequest("GET", "/a", dport=d, ingress=i) for d in (80, 0, 9999) for i in (True, False)]
    reqs.append(L.HTTPRequest("GET", "/a", policy=1))
    arena, offs = L.pack_http(reqs)
    assert HttpProgram(rs.program()).eval(arena, offs).tolist() == [0] * 6 + [L.VERDICT_DENY]


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_random_policy_maps_match_oracle(seed):
    pols = random_policies(seed)
    rs = L.RuleSet.compile_http_policies(pols)
    arena, offs = L.pack_http(random_requests(seed, 600))
    got = HttpProgram(rs.program()).eval(arena, offs)
    exp = PolicyOracle(pols).eval(arena, offs)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    assert len(set(exp.tolist())) > 3
