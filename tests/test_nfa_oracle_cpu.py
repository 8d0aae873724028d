"""The long-input oracle (oracle/nfa.h): a Thompson-NFA /
Pike-VM simulator of the ECMAScript regular subset, independent of the
product's regex front end.  Pinned three ways before config 5 trusts it:
  1. differential fuzz against std::regex_match / regex_search (the engine
     Envoy applies, envoy/cilium_network_policy.h:68-71): random grammar
     patterns x short subjects, syntax acceptance, nested-quantifier families,
     and 1 - 8 KiB subjects on families the backtracker can still finish;
  2. the reference's own known answers (tests/golden/http_known_answers.json)
     through the NFA engine;
  3. constructed long-field truths for config 5's families (paths and values
     up to 64 KiB, tests/adversarial_cases.py), where std::regex backtracks
     exponentially or overflows its stack."""
import os
import subprocess

import numpy as np
import pytest

from cilium_amd import l7match as L
from cilium_amd import workloads as W
import adversarial_cases as A
import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def fuzz_exe(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("nfa") / "fuzz_nfa")
    subprocess.check_call(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "cpp", "fuzz_nfa.cc"), "-o", exe])
    return exe


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_nfa_vs_std_regex_differential_fuzz(fuzz_exe, seed):
    out = subprocess.run([fuzz_exe, str(seed), "3000", "60", "150"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr[-3000:]
    checked = int(out.stdout.split()[1])
    assert checked > 150_000, out.stdout


def test_nfa_known_answers():
    # route.pb.go:2426-2430 (\d{3}) and config-5 style cases, std vs NFA
    cases = [(r"\d{3}", b"123", 1), (r"\d{3}", b"1234", 0), (r"\d{3}", b"123.456", 0),
             (".*public$", b"/maybe/public", 1), (".*REGEX.*", b"hostREGEXname", 1),
             ("(a|aa)*b", b"a" * 30 + b"b", 1), ("(a|aa)*b", b"a" * 30 + b"c", 0),
             ("(.{0,8}){1,8}foo", b"x" * 64 + b"foo", 1), ("(.{0,8}){1,8}foo", b"x" * 65 + b"foo", 0),
             ("(.{0,8}){1,8}foo", b"x\nfoo", 0), (".", b"\r", 0), ("[^]", b"\n", 1), ("[]", b"", 0)]
    for pat, s, want in cases:
        assert O.nfa_match(pat, s) == want, (pat, s[:20])
        if len(s) < 40:
            assert O.regex_match(pat, s) == want, (pat, s)
    assert O.nfa_match("(a)\\1", b"aa") == -2  # back-references: outside the regular subset
    assert O.nfa_match("(?=a)a", b"a") == -2
    assert O.nfa_match("a{2,1}", b"aa") == -1


def test_nfa_long_subjects_linear():
    # 64 KiB subjects the backtracker cannot take (.*b|.* segfaults at 100 KB)
    s = b"a" * 65535
    assert O.nfa_match(".*b|.*", s) == 1
    assert O.nfa_match("(a|aa)*b", s) == 0
    assert O.nfa_match("(a|aa)*", s) == 1
    assert O.nfa_match("[a-z]*[a-z]*[a-z]*[a-z]*z", s + b"z") == 1


def test_http_known_answers_through_nfa_engine():
    from test_http_cpu import _basic_policy_batch, _req, _rule, golden
    for c in golden("http_known_answers.json")["regex_doc"]["cases"]:
        assert O.nfa_match(c["regex"], c["value"].encode()) == int(c["match"])
    g, rules, reqs = _basic_policy_batch()
    arena, offs = L.pack_http(reqs)
    v = O.HttpOracle(rules, engine="nfa").eval(arena, offs)
    assert [bool(x >= 0) for x in v] == [c["allow"] for c in g["cases"]]
    for key in ("readme", "example_http"):
        gg = golden("http_known_answers.json")[key]
        arena, offs = L.pack_http([_req(c["req"]) for c in gg["cases"]])
        v = O.HttpOracle([_rule(r) for r in gg["rules"]], engine="nfa").eval(arena, offs)
        assert v.tolist() == [c["verdict"] for c in gg["cases"]], key


def test_nfa_engine_agrees_on_baseline_configs():
    for cfg, nq in ((1, 3000), (2, 1500)):
        rules = W.rules(cfg)
        arena, offs = W.requests(cfg, 123, nq)
        a = O.HttpOracle(rules, engine="nfa").eval(arena, offs, threads=8)
        b = O.HttpOracle(rules).eval(arena, offs, threads=8)
        assert np.array_equal(a, b), cfg
        assert (a >= 0).any() and (a < 0).any()


def test_config5_nfa_agrees_with_std_regex_where_it_finishes():
    rules = W.rules(5, n_rules=2000)
    arena, offs = W.requests(5, 99, 1500, n_rules=2000)
    a2, o2 = A.subset(arena, offs, A.cheap_for_oracle(arena, offs))
    a = O.HttpOracle(rules, engine="nfa").eval(a2, o2, threads=8)
    b = O.HttpOracle(rules).eval(a2, o2, threads=8)
    assert np.array_equal(a, b)
    assert (a >= 0).sum() > len(a) // 4


def test_config5_constructed_long_fields():
    rules = W.rules(5, n_rules=10_000)
    o = O.HttpOracle(rules, engine="nfa")
    cases = A.long_field_cases(rules, 300) + A.blob_cases(rules, 80)
    arena, offs = L.pack_http([c[0] for c in cases])
    exp = np.array([c[1] for c in cases], dtype=np.int32)
    v = o.eval(arena, offs, threads=8)
    bad = np.nonzero(v != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(v[i])) for i in bad[:10]]
    assert 0.25 < (exp >= 0).mean() < 0.75
    assert max(len(c[0].path) for c in cases) > 60000
