"""GPU parity of HTTP rules with the ECMAScript constructs beyond the regular
core that the reference accepts (std::regex via Envoy,
envoy/cilium_network_policy.h:52-56; verbatim patterns from
pkg/envoy/server.go:276-289): \\b / \\B and look-ahead (exact automata) and
back-references (superset automata + the slow pass, http_slow_kernel running
regex_vm.h), against std::regex_match (oracle/l7oracle.cc), at config-2
scale and on random rule sets."""
import numpy as np
import pytest

import regex_ext_cases as X
from cilium_amd import l7match as L
from cilium_amd import workloads as W
from oracle import ENVOY_THREAD_STACK, HttpOracle
from program_interp import HttpProgram

pytestmark = pytest.mark.gpu


def _check(rules, arena, offs, hits=True):
    rs = L.RuleSet.compile_http(rules)
    h = np.zeros(rs.n_counters, dtype=np.uint64) if hits else None
    got = rs.eval(arena, offs, h)
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    if hits:
        assert int(h[0]) == int((exp == -1).sum())
        for r in np.unique(exp[exp >= 0])[:64]:
            assert int(h[2 + r]) == int((exp == r).sum())
        assert int(h.sum()) == len(exp)
    return got


def test_config2_scale_with_extended_rules(gpu):
    """BASELINE config 2's 1000 rules with the realistic \\b / look-ahead /
    back-reference rules in front of them (indices 0..9, so they decide
    first), over 200k config-2 requests plus requests aimed at them."""
    rng = np.random.default_rng(42)
    rules = list(X.REALISTIC) + W.rules(2)
    a1, o1 = W.requests(2, 3_000_000, 200_000)
    reqs = X.realistic_requests(rng, 20_000) + X.random_requests(rng, 10_000)
    a2, o2 = L.pack_http(reqs)
    arena = np.concatenate([a1[:-64], a2])
    offs = np.concatenate([o1, o2 + np.uint64(len(a1) - 64)])
    got = _check(rules, arena, offs)
    assert {0, 1, 2, 8, 9} <= set(got.tolist())
    assert (got >= len(X.REALISTIC)).sum() > 10_000  # config-2 rules still decide most


def test_random_extended_rule_sets(gpu):
    rng = np.random.default_rng(7)
    for trial in range(24):
        rules = X.random_rules(rng, int(rng.integers(1, 24)), backrefs=trial % 2 == 1)
        arena, offs = L.pack_http(X.random_requests(rng, 4000))
        _check(rules, arena, offs)


def test_slow_path_decides_what_the_reference_decides(gpu):
    """Long subjects through back-reference rules: the GPU (two-tier slow pass,
    regex_vm.h) against std::regex_match itself, run by the oracle on a
    measured 1 GiB stack.  Every request whose reference evaluation fits an
    8 MiB thread stack (an Envoy worker's) gets the reference's verdict; −3
    appears only where the oracle measured more than 8 MiB of native stack,
    i.e. where std::regex_match would overflow the worker and crash Envoy."""
    # rule 0 (4 executor words per byte) decides the b-runs; the c-runs reach
    # rule 1 (16 words per byte, 834 native bytes per byte in libstdc++)
    rules = [L.PortRuleHTTP(Path="/(a)(?:b)*\\1z"), L.PortRuleHTTP(Path="/(a)(b|c)*\\1z"),
             L.PortRuleHTTP(Path="/.*")]
    sizes = (10, 100, 2000, 8000, 12000, 20000, 40000, 60000)
    reqs = [L.HTTPRequest("GET", "/a" + "b" * n + "az") for n in sizes]
    reqs += [L.HTTPRequest("GET", "/a" + "b" * n + "ay") for n in sizes]  # rule 2 decides
    reqs += [L.HTTPRequest("GET", "/a" + "c" * n + "az") for n in (2000, 8000, 12000, 20000, 40000)]
    arena, offs = L.pack_http(reqs)
    rs = L.RuleSet.compile_http(rules)
    got = rs.eval(arena, offs)
    exp, used = HttpOracle(rules, prefilter=False).eval_stack(arena, offs)
    decided_long = 0
    for i in range(len(reqs)):
        if used[i] <= ENVOY_THREAD_STACK:
            assert got[i] == exp[i], (i, int(got[i]), int(exp[i]), int(used[i]))
        elif got[i] != L.VERDICT_UNSUPPORTED:
            assert got[i] == exp[i], (i, int(got[i]), int(exp[i]), int(used[i]))
            decided_long += 1
        if got[i] == L.VERDICT_UNSUPPORTED:
            assert used[i] > ENVOY_THREAD_STACK, (i, int(used[i]))
    assert got[:6].tolist() == [0] * 6  # n = 8 k, 12 k, 20 k decided (round 4: -3 from 12 k)
    assert decided_long > 0 and L.VERDICT_UNSUPPORTED in got.tolist()
    assert got.tolist() == HttpProgram(rs.program()).eval(arena, offs).tolist()


def test_extended_rules_slow_pass_share(gpu):
    """bench.py --extended's workload: config 2 with the extended rules in
    front.  The back-reference rule whose superset automaton matches most
    config-2 paths (/(\\w+)/\\1(/.*)?) is a forced capture decided in the
    first pass (program.h DcapSpec); no verdict is −3."""
    rules = list(X.REALISTIC) + W.rules(2)
    arena, offs = W.requests(2, 5_000_000, 300_000, n_rules=1000)
    got = _check(rules, arena, offs)
    assert L.VERDICT_UNSUPPORTED not in got.tolist()


def test_forced_capture_backreferences(gpu):
    """Back-references whose capture is forced (regex_ecma.h DcapForm) are
    decided in the first pass by byte compares; near-miss forms keep the slow
    pass.  GPU verdicts and counters against std::regex_match, in front of
    config 2's rules and alone."""
    rng = np.random.default_rng(62)
    for trial in range(8):
        rules = X.dcap_rules(rng, int(rng.integers(2, 16)))
        if trial % 2:
            rules = rules + W.rules(2, n_rules=300)
        arena, offs = L.pack_http(X.dcap_requests(rng, 20_000))
        got = _check(rules, arena, offs)
        assert (got >= 0).any()


def test_step_budget_outcomes_pinned_against_the_oracle(gpu):
    """The executor's step budgets (regex_vm.h: tier 1 2^22, tier 2 2^25
    steps) on exponential backtracking the first pass cannot rule out:
    /((a|a)*)c\\1d over /a^n c a^(n+1) d.  The superset automaton accepts
    (the reference group becomes a^*), and std::regex (no step limit) tries
    all 2^n ways to match a^n before it fails, so rule 1 allows every n.
    The GPU equals it wherever the host build of the executor decides within
    the tier-2 budget, and answers -3 (L7M_VERDICT_UNSUPPORTED) exactly where
    that budget runs out -- never a wrong allow or deny."""
    import time
    from program_interp import _VM, VM_SCRATCH_WORDS, VM_MAX_STEPS, VM_LIMIT
    pat = "/((a|a)*)c\\1d"
    rules = [L.PortRuleHTTP(Path=pat), L.PortRuleHTTP(Path="/.*")]
    sizes = list(range(12, 25, 2))
    subj = ["/" + "a" * n + "c" + "a" * (n + 1) + "d" for n in sizes]
    reqs = [L.HTTPRequest("GET", x) for x in subj]
    arena, offs = L.pack_http(reqs)
    rs = L.RuleSet.compile_http(rules)
    got = rs.eval(arena, offs)
    t0 = time.perf_counter()
    exp = HttpOracle(rules, prefilter=False).eval(arena, offs)
    assert time.perf_counter() - t0 < 120
    P = HttpProgram(rs.program())
    h = P.h
    assert h["n_slow"] == 1 and not P.dcaps  # a loop inside the group: not a forced capture
    so, _ = P.w[h["off_slow"]: h["off_slow"] + 2]
    prog = P.prog[P.w[h["off_pool"] + so + 1]:]
    limited = []
    for i, n in enumerate(sizes):
        s = subj[i].encode()
        r = _VM.vm_host_match(prog.ctypes.data, s, len(s), VM_SCRATCH_WORDS, VM_MAX_STEPS)
        assert exp[i] == 1  # the reference decides: rule 0 fails, rule 1 allows
        if r == VM_LIMIT:
            limited.append(n)
            assert got[i] == L.VERDICT_UNSUPPORTED, (n, int(got[i]))
        else:
            assert got[i] == exp[i], (n, int(got[i]))
    assert limited and limited[0] > sizes[0]  # the budget runs out only past n ~ 22
    assert got.tolist() == P.eval(arena, offs).tolist()
