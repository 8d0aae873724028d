"""NPDS policy maps on the GPU: the kernel's port-entry selection
(exact port, port 0, no entry, entries without HTTP rules, unknown endpoint
policy, ingress vs egress) bit-exact against the NetworkPolicyMap oracle,
including the reference's ingress and egress integration cases
(envoy/cilium_integration_test.cc:605-717)."""
import numpy as np
import pytest

from cilium_amd import l7match as L
from oracle import PolicyOracle
from policy_cases import basic_requests, golden_npds, npds, random_policies, random_requests

pytestmark = pytest.mark.gpu


def test_npds_known_answers_gpu(gpu):
    g = golden_npds()
    pols = [npds(g["policy"])]
    reqs, expect = basic_requests(g)
    m = L.NetworkPolicyMap(pols)
    allowed = m.Allowed(reqs, ["173"] * len(reqs))
    assert allowed.tolist() == expect
    # a name the map does not hold: Allowed() is false (h:231-235)
    assert not m.Allowed(reqs, ["174"] * len(reqs)).any()


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_random_policy_maps_gpu(gpu, seed):
    pols = random_policies(seed, n_policies=4)
    rs = L.RuleSet.compile_http_policies(pols)
    arena, offs = L.pack_http(random_requests(seed, 20000, n_policies=4))
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    got = rs.eval(arena, offs, h)
    exp = PolicyOracle(pols).eval(arena, offs, threads=8)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    # counters: denies + per-rule allows (allow-without-rule verdicts are not counted)
    counted = int(((got >= 0) & (got < L.VERDICT_ALLOW_NO_PORT_POLICY)).sum()) + int((got == -1).sum())
    assert int(h.sum()) == counted
