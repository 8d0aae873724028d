"""CPU tests: C-ABI library surface, oracle pinned to the reference's own known
answers, and the HTTP rule compiler (via tests/program_interp.py) against the
oracle.  No GPU calls."""
import json
import os
import re
import subprocess

import numpy as np
import pytest

import regex_ext_cases as X

from cilium_amd import l7match as L
from cilium_amd import workloads as W
from oracle import HttpOracle, OracleError, regex_match
from program_interp import HttpProgram

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def golden(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def _rule(d):
    return L.PortRuleHTTP(Path=d.get("Path", ""), Method=d.get("Method", ""), Host=d.get("Host", ""),
                          Headers=d.get("Headers", []), RemoteIDs=d.get("RemoteIDs", []))


def _req(d, **kw):
    return L.HTTPRequest(method=d.get("method"), path=d.get("path"), authority=d.get("authority", "host"),
                         headers=[tuple(h) for h in d.get("headers", [])], **kw)


# ---------------------------------------------------------------- C ABI ----
def test_library_exports_every_header_symbol():
    hdr = open(os.path.join(ROOT, "include", "l7match.h")).read()
    declared = sorted(set(re.findall(r"\b(l7m_[a-z_]+)\s*\(", hdr)))
    assert declared, "no declarations parsed"
    lib = L.lib()
    for sym in declared:
        assert hasattr(lib, sym), f"libl7match.so does not export {sym}"
    assert set(declared) == set(L.EXPORTED_SYMBOLS)
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    for sym in declared:
        assert re.search(rf"\bT {sym}\b", out), sym
    assert lib.l7m_abi_version() == 4


def test_eval_without_device_fails_loudly():
    if L.device_count() > 0:
        pytest.skip("GPU present")
    rs = L.RuleSet.compile_http([L.PortRuleHTTP(Path="/a")])
    arena, offs = L.pack_http([L.HTTPRequest("GET", "/a")])
    with pytest.raises(L.L7Error) as e:
        rs.eval(arena, offs)
    assert e.value.code == L.L7M_EDEVICE


# ------------------------------------------------------ translation (A1) ----
def test_get_http_rule_translation_known_answers():
    for case in golden("http_known_answers.json")["translation"]["cases"]:
        got = L.get_http_rule(_rule(case["rule"]))
        exp = [L.HeaderMatcher(m["Name"], m["Value"], m["Regex"]) for m in case["expected"]]
        assert got == exp


def test_header_spec_splitting():
    got = L.get_http_rule(L.PortRuleHTTP(Headers=["X-Token:: a b", "X-Only", "Colon: "]))
    names = {(m.Name, m.Value, m.kind) for m in got}
    assert ("X-Token", "a b", "value") in names       # SplitN(h, " ", 2), TrimRight ":"
    assert ("X-Only", "", "present") in names
    assert ("Colon", "", "present") in names          # empty literal value -> presence


def test_duplicate_header_matcher_is_rejected_like_go_sort_panic():
    with pytest.raises(L.L7Error) as e:
        L.RuleSet.compile_http([L.PortRuleHTTP(Headers=["X-A: 1", "X-A: 1"])])
    assert e.value.code == L.L7M_EINVAL_RULE
    with pytest.raises(L.L7Error):
        L.RuleSet.compile_http([L.PortRuleHTTP(Path="/x", Headers=[":path /x"])])
    # distinct case in the name is not a Go-equal pair
    L.RuleSet.compile_http([L.PortRuleHTTP(Headers=["X-A: 1", "x-a: 1"])])


def test_invalid_regex_nacks_and_unsupported_is_explicit():
    for bad in ("a{,3}", "(?i)abc", "[z-a]", "a{2,1}", "*a", "(", "[\\d-z]"):
        with pytest.raises(L.L7Error) as e:
            L.RuleSet.compile_http([L.PortRuleHTTP(Path=bad)])
        assert e.value.code == L.L7M_EINVAL_REGEX, bad
        with pytest.raises(OracleError):
            HttpOracle([L.PortRuleHTTP(Path=bad)])
    # \\b, \\B and look-ahead compile (exact automata, regex_ecma.cc build_ctx)
    for ok in ("\\bfoo", "(?=a)a", "a(?!b)", "x\\B"):
        L.RuleSet.compile_http([L.PortRuleHTTP(Path=ok)])


def test_word_boundary_lookahead_and_backreference_rules_match_oracle():
    """Realistic and random rule sets with \\b / \\B / (?=) / (?!) (exact
    automata) and back-references (superset automata + the slow path, whose
    executor runs here through its host build) through the program
    interpreter (the kernel's two passes) against std::regex_match."""
    rng = np.random.default_rng(5)
    reqs = X.realistic_requests(rng, 3000) + X.random_requests(rng, 2000)
    arena, offs = L.pack_http(reqs)
    v = _interp_vs_oracle(X.REALISTIC, arena, offs)
    assert len(set(v.tolist())) >= 8
    assert {8, 9} <= set(v.tolist())  # the back-reference rules decide some requests
    for trial in range(16):
        rules = X.random_rules(rng, int(rng.integers(1, 16)), backrefs=trial % 2 == 1)
        arena, offs = L.pack_http(X.random_requests(rng, 1500))
        _interp_vs_oracle(rules, arena, offs)


def test_forced_capture_backreferences_first_pass_match_oracle():
    """Back-references whose capture is forced (regex_ecma.h DcapForm, e.g.
    bench.py --extended's /(\\w+)/\\1(/.*)?) are decided in the first pass by
    byte compares (program.h DcapSpec) instead of the slow path; near-miss
    forms keep the slow path.  The program interpreter (the kernel's
    algorithm) equals std::regex_match on paths built to hit and miss them."""
    rng = np.random.default_rng(61)
    n_dcap = n_slow = 0
    for trial in range(12):
        rules = X.dcap_rules(rng, int(rng.integers(1, 12)))
        prog = HttpProgram(L.RuleSet.compile_http(rules).program())
        n_dcap += len(prog.dcaps)
        n_slow += prog.h["n_slow"]
        arena, offs = L.pack_http(X.dcap_requests(rng, 1500))
        v = _interp_vs_oracle(rules, arena, offs)
        assert (v >= 0).any()
    assert n_dcap > 20 and n_slow > 0
    # the extended rules' /(\\w+)/\\1(/.*)? leaves the slow path
    prog = HttpProgram(L.RuleSet.compile_http(X.REALISTIC).program())
    assert len(prog.dcaps) == 1 and prog.h["n_slow"] == 1


def test_forced_capture_analysis_differential_fuzz():
    """tests/cpp/fuzz_dcap.cc: random P1 (C{n,m}) L2 \\1 R patterns and near
    misses; wherever regex_ecma.h analyze_dcap accepts one, the first-pass
    decision (P1, maximal class run, L2, the run repeated, R's automaton)
    equals std::regex_match on every subject."""
    exe = "/tmp/l7m_fuzz_dcap"
    src = os.path.join(ROOT, "tests", "cpp", "fuzz_dcap.cc")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-o", exe, src,
                           os.path.join(ROOT, "cilium_amd", "csrc", "regex_ecma.cc"),
                           os.path.join(ROOT, "cilium_amd", "csrc", "dfa_pack.cc"),
                           os.path.join(ROOT, "cilium_amd", "csrc", "regex_vm.cc")])
    for seed in ("5", "6"):
        out = subprocess.run(["timeout", "240", exe, seed, "2000", "200"], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout[-3000:]
        assert "mismatches=0" in out.stdout


def test_unknown_dialect_is_rejected():
    with pytest.raises(L.L7Error) as e:
        L.RuleSet.compile_http([L.PortRuleHTTP(Path="/a")], dialect=7)
    assert e.value.code == L.L7M_EINVAL


# ------------------------------------------------- oracle vs known answers --
def test_oracle_regex_doc_examples():
    for c in golden("http_known_answers.json")["regex_doc"]["cases"]:
        assert regex_match(c["regex"], c["value"].encode()) == int(c["match"])


def _basic_policy_batch():
    g = golden("http_known_answers.json")["basic_policy"]
    rules = [_rule(r) for r in g["rules"]]
    reqs = [L.HTTPRequest(c["method"], c["path"], c["authority"], remote_id=g["remote_id"], dport=g["dport"])
            for c in g["cases"]]
    return g, rules, reqs


def test_oracle_envoy_integration_known_answers():
    g, rules, reqs = _basic_policy_batch()
    arena, offs = L.pack_http(reqs)
    v = HttpOracle(rules).eval(arena, offs)
    for c, x in zip(g["cases"], v):
        assert (x >= 0) == c["allow"], c["name"]


@pytest.mark.parametrize("key", ["readme", "example_http"])
def test_oracle_readme_and_example_known_answers(key):
    g = golden("http_known_answers.json")[key]
    rules = [_rule(r) for r in g["rules"]]
    arena, offs = L.pack_http([_req(c["req"]) for c in g["cases"]])
    v = HttpOracle(rules).eval(arena, offs)
    assert v.tolist() == [c["verdict"] for c in g["cases"]]


# ---------------------------------------------- compiler vs oracle (CPU) --
def _interp_vs_oracle(rules, arena, offs):
    rs = L.RuleSet.compile_http(rules)
    got = HttpProgram(rs.program()).eval(arena, offs)
    exp = HttpOracle(rules).eval(arena, offs)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    return exp


def test_compiler_known_answers():
    g, rules, reqs = _basic_policy_batch()
    arena, offs = L.pack_http(reqs)
    v = _interp_vs_oracle(rules, arena, offs)
    assert [(x >= 0) for x in v] == [c["allow"] for c in g["cases"]]
    for key in ("readme", "example_http"):
        gg = golden("http_known_answers.json")[key]
        arena, offs = L.pack_http([_req(c["req"]) for c in gg["cases"]])
        _interp_vs_oracle([_rule(r) for r in gg["rules"]], arena, offs)


@pytest.mark.parametrize("cfg,n", [(1, 4000), (2, 4000)])
def test_compiler_vs_oracle_on_baseline_configs(cfg, n):
    rules = W.rules(cfg)
    arena, offs = W.requests(cfg, 1_000_000, n)
    v = _interp_vs_oracle(rules, arena, offs)
    assert (v >= 0).any() and (v == -1).any()


def test_compiler_group_splitting_matches_single_group():
    rules = W.rules(2, n_rules=200)
    arena, offs = W.requests(2, 0, 2000, n_rules=200)
    rs_small = L.RuleSet.compile_http(rules, max_dfa_states=16)
    assert rs_small.info.n_dfas > L.RuleSet.compile_http(rules).info.n_dfas
    got = HttpProgram(rs_small.program()).eval(arena, offs)
    exp = HttpOracle(rules).eval(arena, offs)
    assert (got == exp).all()


@pytest.mark.parametrize("budget", [1, 4096])
def test_compiler_hbm_resident_tables_match_oracle(budget):
    """Tables that do not fit the LDS budget are walked from HBM (u32 copies)."""
    rules = W.rules(2, n_rules=150)
    arena, offs = W.requests(2, 0, 1500, n_rules=150)
    rs = L.RuleSet.compile_http(rules, lds_budget_bytes=budget)
    P = HttpProgram(rs.program())
    assert any(d["lds_table"] == 0xFFFFFFFF for d in P.dfas)
    assert (P.eval(arena, offs) == HttpOracle(rules).eval(arena, offs)).all()


def test_compiler_edge_cases():
    rules = [
        L.PortRuleHTTP(Headers=["X-Dup"]),                 # presence-only rule
        L.PortRuleHTTP(Path="", Method="", Host=""),       # empty rule: matches everything
    ]
    reqs = [L.HTTPRequest("GET", "/", None, []), L.HTTPRequest("GET", "/", "h", [("x-dup", "a"), ("x-dup", "b")])]
    arena, offs = L.pack_http(reqs)
    assert _interp_vs_oracle(rules, arena, offs).tolist() == [1, 0]
    # empty rule list: no L7 rules on the port -> allow (cilium_network_policy.h:129-135)
    assert _interp_vs_oracle([], arena, offs).tolist() == [L.VERDICT_ALLOW_NO_L7] * 2
    # first occurrence of a repeated header decides; absent authority fails ':authority' matchers
    rules = [L.PortRuleHTTP(Headers=["X-Dup: b"]), L.PortRuleHTTP(Host=".*"), L.PortRuleHTTP(Headers=["X-Dup: a"])]
    assert _interp_vs_oracle(rules, arena, offs).tolist() == [-1, 1]
    # remote-id restricted rule without matchers
    rules = [L.PortRuleHTTP(RemoteIDs=[7])]
    reqs = [L.HTTPRequest("GET", "/", remote_id=7), L.HTTPRequest("GET", "/", remote_id=8)]
    arena, offs = L.pack_http(reqs)
    assert _interp_vs_oracle(rules, arena, offs).tolist() == [0, -1]


def test_regex_compiler_differential_fuzz():
    """Build and run tests/cpp/fuzz_regex.cc: the ECMAScript parser + DFA
    builder against std::regex_match on random patterns and inputs."""
    exe = "/tmp/l7m_fuzz_regex"
    src = os.path.join(ROOT, "tests", "cpp", "fuzz_regex.cc")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-o", exe, src,
                           os.path.join(ROOT, "cilium_amd", "csrc", "regex_ecma.cc"),
                           os.path.join(ROOT, "cilium_amd", "csrc", "dfa_pack.cc"),
                           os.path.join(ROOT, "cilium_amd", "csrc", "regex_vm.cc")])
    out = subprocess.run(["timeout", "240", exe, "7", "600", "120"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout[-3000:]
    assert "mismatches=0" in out.stdout
    # word boundaries, look-ahead (exact) and back-references (superset automata)
    for seed in ("11", "12"):
        out = subprocess.run(["timeout", "240", exe, seed, "3000", "100", "1"], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout[-3000:]
        assert "mismatches=0" in out.stdout and "packed_mismatch=0" in out.stdout


def test_compiler_table_only_lds_placement_matches_oracle():
    """A slot table that fits the LDS budget only without its u16 end codes /
    latches is placed alone (end codes stay in the program)."""
    rules = W.rules(2, n_rules=400)
    arena, offs = W.requests(2, 0, 1500, n_rules=400)
    found = False
    for budget in range(8192, 24576, 512):  # a budget where one table fits only without its end codes
        P = HttpProgram(L.RuleSet.compile_http(rules, lds_budget_bytes=budget).program())
        if any(d["lds_table"] != 0xFFFFFFFF and d["lds_es"] == 0xFFFFFFFF for d in P.dfas):
            found = True
            break
    assert found
    assert (P.eval(arena, offs) == HttpOracle(rules).eval(arena, offs)).all()


@pytest.mark.parametrize("cfg,n_rules", [(2, 1000), (1, None), (5, 400)])
def test_verification_masks_match_candidate_tables(cfg, n_rules):
    """The header's cand_dfas / pres_fields masks (the kernel's uniform skips
    in verification) name exactly the DFAs with candidate entries and the
    fields with presence-keyed check records."""
    rules = W.rules(cfg, n_rules=n_rules) if n_rules else W.rules(cfg)
    P = HttpProgram(L.RuleSet.compile_http(rules).program())
    h = P.h
    cand = h["cand_dfas_lo"] | h["cand_dfas_hi"] << 32
    pres = h["pres_fields_lo"] | h["pres_fields_hi"] << 32
    for k in range(h["n_dfas"]):
        d = P.dfas[k]
        n_ct = d["nsets"] + d["npats"]
        has = any(P.w[d["ct_off"] + 16 * i] for i in range(n_ct))
        assert bool(cand >> k & 1) == has, k
    for f, fd in enumerate(P.fields):
        assert bool(pres >> f & 1) == (fd[3] > 0), f
    assert cand != 0


def test_nul_and_high_bytes_in_fields_interpreter():
    """The program interpreter (LDS image encoding: zero dead row, byte-address
    rows) on fields with NUL and high bytes equals std::regex."""
    import raw_cases
    rules, arena, offs = raw_cases.nul_high_byte_case(1500)
    exp = HttpOracle(rules).eval(arena, offs)
    got = HttpProgram(L.RuleSet.compile_http(rules).program()).eval(arena, offs)
    assert np.array_equal(got, exp)
    assert (exp >= 0).any() and (exp == -1).any()
