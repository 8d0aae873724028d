"""GPU parity tests: HTTP verdicts of the HIP kernel (through the C ABI) versus
the CPU oracle, bit-exact (int32 verdict = deny / first matching rule)."""
import json
import os

import numpy as np
import pytest

from cilium_amd import l7match as L
from cilium_amd import workloads as W
from oracle import HttpOracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def golden(name):
    with open(os.path.join(ROOT, "tests", "golden", name)) as f:
        return json.load(f)


def _rule(d):
    return L.PortRuleHTTP(Path=d.get("Path", ""), Method=d.get("Method", ""), Host=d.get("Host", ""),
                          Headers=d.get("Headers", []), RemoteIDs=d.get("RemoteIDs", []))


def _check(rules, arena, offs, hits=False):
    rs = L.RuleSet.compile_http(rules)
    h = np.zeros(rs.n_counters, dtype=np.uint64) if hits else None
    got = rs.eval(arena, offs, h)
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    if hits:
        assert int(h[0]) == int((exp == -1).sum())
        assert int(h[1]) == int((exp <= -2).sum())
        for r in np.unique(exp[exp >= 0])[:50]:
            assert int(h[2 + r]) == int((exp == r).sum())
        assert int(h.sum()) == len(exp)
    return got


def test_envoy_integration_known_answers(gpu):
    g = golden("http_known_answers.json")["basic_policy"]
    rules = [_rule(r) for r in g["rules"]]
    reqs = [L.HTTPRequest(c["method"], c["path"], c["authority"], remote_id=g["remote_id"], dport=g["dport"])
            for c in g["cases"]]
    arena, offs = L.pack_http(reqs)
    v = _check(rules, arena, offs)
    assert [bool(x >= 0) for x in v] == [c["allow"] for c in g["cases"]]
    # the remote-2-only rule allows identity 2 (L3DeniedPath's counterpart)
    arena, offs = L.pack_http([L.HTTPRequest("GET", "/only-2-allowed", "host", remote_id=2)])
    assert _check(rules, arena, offs).tolist() == [5]


@pytest.mark.parametrize("key", ["readme", "example_http"])
def test_readme_and_example_known_answers(gpu, key):
    g = golden("http_known_answers.json")[key]
    reqs = [L.HTTPRequest(c["req"]["method"], c["req"]["path"], "host",
                          [tuple(h) for h in c["req"]["headers"]]) for c in g["cases"]]
    arena, offs = L.pack_http(reqs)
    v = _check([_rule(r) for r in g["rules"]], arena, offs)
    assert v.tolist() == [c["verdict"] for c in g["cases"]]


@pytest.mark.parametrize("cfg,n", [(1, 200_000), (2, 100_000)])
def test_baseline_config_sample_parity(gpu, cfg, n):
    rules = W.rules(cfg)
    arena, offs = W.requests(cfg, 5_000_000, n)
    v = _check(rules, arena, offs, hits=True)
    assert (v >= 0).any() and (v == -1).any()


def test_group_split_parity(gpu):
    rules = W.rules(2, n_rules=300)
    arena, offs = W.requests(2, 0, 20_000, n_rules=300)
    rs = L.RuleSet.compile_http(rules, max_dfa_states=16)
    assert rs.info.n_dfas > L.RuleSet.compile_http(rules).info.n_dfas
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    assert (rs.eval(arena, offs) == exp).all()


def test_edge_cases(gpu):
    rules = [L.PortRuleHTTP(Headers=["X-Dup: b"]), L.PortRuleHTTP(Host=".*"),
             L.PortRuleHTTP(Headers=["X-Dup: a"]), L.PortRuleHTTP(Path="/(a|b)*c{2,3}$", Method="[A-Z]{3,}")]
    long_val = "a" * 65535
    reqs = [
        L.HTTPRequest("GET", "/", None, []),
        L.HTTPRequest("GET", "/", None, [("x-dup", "a"), ("x-dup", "b")]),
        L.HTTPRequest("GET", "/", None, [("x-dup", "b"), ("x-dup", "a")]),
        L.HTTPRequest("GET", "/", "", []),
        L.HTTPRequest("POST", "/ababcc", None, []),
        # std::regex (the oracle) recurses per character: keep regex inputs < 8 KB
        L.HTTPRequest("GET", "/" + "ab" * 3000 + "ccc", None, []),
        L.HTTPRequest("GET", "/abcccc", None, []),
        L.HTTPRequest("GE", "/cc", None, []),
        L.HTTPRequest(None, "/cc", None, []),
        L.HTTPRequest("GET", long_val, None, [("x-dup", long_val)]),
        L.HTTPRequest("GET", "/", None, [("h%d" % k, "v") for k in range(255)]),
        L.HTTPRequest("GET", "/", None, [("h%d" % k, "v") for k in range(254)] + [("x-dup", "a")]),
    ]
    arena, offs = L.pack_http(reqs)
    v = _check(rules, arena, offs, hits=True)
    assert v.tolist() == [-1, 2, 0, 1, 3, 3, -1, -1, -1, -1, -1, 2]


def test_empty_batch_and_empty_ruleset(gpu):
    rs = L.RuleSet.compile_http([L.PortRuleHTTP(Path="/a")])
    v = rs.eval(np.zeros(64, np.uint8), np.zeros(0, np.uint64))
    assert v.shape == (0,)
    arena, offs = L.pack_http([L.HTTPRequest("GET", "/x")] * 3)
    assert L.RuleSet.compile_http([]).eval(arena, offs).tolist() == [L.VERDICT_ALLOW_NO_L7] * 3


def test_malformed_records_report_parse_error(gpu):
    arena, offs = L.pack_http([L.HTTPRequest("GET", "/a", "h", [("x", "y")])] * 4)
    arena = arena.copy()
    rec = int(offs[1])
    arena[rec:rec + 4] = np.frombuffer(np.uint32(999).tobytes(), np.uint8)   # wrong rec_len
    offs = offs.copy()
    offs[2] = arena.nbytes + 4096                                           # outside the arena
    offs[3] = offs[3] + 2                                                   # misaligned
    rules = [L.PortRuleHTTP(Path="/a")]
    v = L.RuleSet.compile_http(rules).eval(arena, offs)
    assert v.tolist() == [0, L.VERDICT_PARSE_ERROR, L.VERDICT_PARSE_ERROR, L.VERDICT_PARSE_ERROR]


def test_random_regex_rules_parity(gpu):
    """Random small regex rule sets over random requests (oracle = std::regex)."""
    rng = np.random.default_rng(11)
    atoms = ["a", "b", "/", ".", "[a-c]", "[^/]", "\\d", "\\w", "(x|yz)", "[0-9]{1,3}", "-"]
    for trial in range(20):
        rules = []
        for _ in range(int(rng.integers(1, 12))):
            def pat():
                s = "".join(rng.choice(atoms) + rng.choice(["", "*", "+", "?", "{0,2}"]) for _ in range(rng.integers(1, 5)))
                return s if rng.random() > 0.1 else "^" + s + "$"
            rules.append(L.PortRuleHTTP(Path=pat() if rng.random() < 0.8 else "",
                                        Method=rng.choice(["", "GET", "GET|POST", "[A-Z]+"]),
                                        Host=pat() if rng.random() < 0.3 else "",
                                        Headers=list(rng.choice(["", "x-a: 1", "x-b"], size=1)) if rng.random() < 0.3 else []))
            rules[-1].Headers = [h for h in rules[-1].Headers if h]
        alpha = list("ab/.-xyz0129c")
        reqs = []
        for _ in range(3000):
            hdrs = []
            if rng.random() < 0.5:
                hdrs.append(("x-a", rng.choice(["1", "2"])))
            if rng.random() < 0.3:
                hdrs.append(("x-b", ""))
            reqs.append(L.HTTPRequest(rng.choice(["GET", "POST", "put"]),
                                      "".join(rng.choice(alpha, size=rng.integers(0, 10))),
                                      "".join(rng.choice(alpha, size=rng.integers(0, 6))), hdrs))
        arena, offs = L.pack_http(reqs)
        _check(rules, arena, offs)


def test_eval_device_matches_host_eval_and_shards(gpu):
    import torch
    rules = W.rules(2)
    rs = L.RuleSet.compile_http(rules)
    arena, offs = W.requests(2, 0, 300_000)
    host_v = rs.eval(arena, offs)
    dev = torch.device("cuda:0")
    da = torch.from_numpy(arena).to(dev)
    do = torch.from_numpy(offs.view(np.int64)).to(dev)
    dv = torch.empty(len(offs), dtype=torch.int32, device=dev)
    dh = torch.zeros(rs.n_counters, dtype=torch.int64, device=dev)
    rs.eval_device(da, arena.nbytes, do, len(offs), dv, dh, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert (dv.cpu().numpy() == host_v).all()
    assert int(dh.sum()) == len(offs)
    # shard invariance: two halves generated independently == one batch
    a1, o1 = W.requests(2, 0, 150_000)
    a2, o2 = W.requests(2, 150_000, 150_000)
    v = np.concatenate([rs.eval(a1, o1), rs.eval(a2, o2)])
    assert (v == host_v).all()


@pytest.mark.parametrize("budget", [1, 8192, 12288, 16384])
def test_lds_placement_variants_parity(gpu, budget):
    """Every LDS placement of the DFA tables — none, full (table + u16 end
    codes), and table-only (end codes read from the program) — gives the
    oracle's verdicts and counters."""
    rules = W.rules(2, n_rules=400)
    arena, offs = W.requests(2, 3_000_000, 20_000, n_rules=400)
    rs = L.RuleSet.compile_http(rules, lds_budget_bytes=budget)
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    got = rs.eval(arena, offs, h)
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    assert int(h.sum()) == len(offs)


@pytest.mark.parametrize("n_fields", [1, 4, 8])
def test_end_code_storage_and_header_jobs(gpu, n_fields):
    """Programs with <= 4, 5-8 and > 8 value DFAs keep end codes in 4
    registers, 8 registers or LDS columns (l7m_kernels.hip Codes<>); header
    jobs skip names of unreferenced lengths, hash the rest, take the first
    occurrence; presence-keyed rules go through the presence mask."""
    rng = np.random.default_rng(7000 + n_fields)
    names = [f"x-h{j}" for j in range(n_fields)]
    rules = []
    for i in range(60):
        hs = []
        for j in rng.choice(n_fields, size=min(n_fields, 1 + int(rng.integers(0, 3))), replace=False):
            hs.append(f"{names[j]}: v{int(rng.integers(0, 4))}" if rng.random() < 0.7 else names[j])
        rules.append(L.PortRuleHTTP(Path=f"/p{i % 7}/.*" if rng.random() < 0.8 else "",
                                    Method=["GET", "POST", ""][i % 3], Headers=hs))
    reqs = []
    for _ in range(3000):
        hs = []
        for _k in range(int(rng.integers(0, 7))):
            r = rng.random()
            if r < 0.6:
                hs.append((names[int(rng.integers(0, n_fields))], f"v{int(rng.integers(0, 5))}"))
            elif r < 0.8:  # an unreferenced name of a referenced length
                hs.append((f"y-h{int(rng.integers(0, 9))}", "v1"))
            else:
                hs.append(("user-agent", "curl/7.88"))
        reqs.append(L.HTTPRequest(["GET", "POST", "PUT"][int(rng.integers(0, 3))],
                                  f"/p{int(rng.integers(0, 9))}/{int(rng.integers(0, 100))}", "h", hs))
    arena, offs = L.pack_http(reqs)
    rs = L.RuleSet.compile_http(rules)
    assert (rs.info.n_dfas <= 4) == (n_fields == 1) and (rs.info.n_dfas > 8) == (n_fields == 8)
    v = _check(rules, arena, offs, hits=True)
    assert (v >= 0).any() and (v == -1).any()



def test_nul_and_high_bytes_in_fields(gpu):
    """Fields holding NUL and high bytes (the LDS walk's dead row is the zero
    row at image address 0, reached by a byte-3 address fold: a NUL byte after
    a dead transition must keep the walk dead, a 0xff byte must not alias):
    verdicts equal std::regex's on random byte strings."""
    import raw_cases
    rules, arena, offs = raw_cases.nul_high_byte_case(4000)
    got = _check(rules, arena, offs)
    assert (got >= 0).any() and (got == -1).any()
