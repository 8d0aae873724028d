"""L7M_DIALECT_RE2_SEARCH (Go regexp MatchString) on CPU: the oracle
(std::regex_search) pinned by tests/golden/re2_search.json (Python re.search
vectors over the intersection grammar + RE2 syntax rules; "RE2-semantics,
not run against Go"), and the RE2 compiler checked through the program
interpreter against the same vectors and the oracle."""
import json
import os

import numpy as np
import pytest

from cilium_amd import l7match as L
from oracle import HttpOracle, regex_search
from program_interp import HttpProgram
from cilium_amd import workloads as W

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "re2_search.json")
RE2 = L.DIALECT_RE2_SEARCH


def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def _by_pattern(cases):
    out = {}
    for c in cases:
        out.setdefault(c["pattern"], []).append((c["subject"].encode("latin-1"), c["match"]))
    return out


def test_oracle_pinned_by_golden_vectors():
    for c in golden()["search"]:
        assert regex_search(c["pattern"], c["subject"].encode("latin-1")) == int(c["match"]), c


def _interp_paths(pattern, subjects):
    rs = L.RuleSet.compile_http([L.PortRuleHTTP(Path=pattern)], dialect=RE2)
    arena, offs = L.pack_http([L.HTTPRequest("GET", s, "h") for s in subjects])
    return HttpProgram(rs.program()).eval(arena, offs)


def test_compiler_matches_golden_search_vectors():
    for pattern, items in _by_pattern(golden()["search"]).items():
        got = _interp_paths(pattern, [s for s, _ in items])
        assert [int(v) == 0 for v in got] == [m for _, m in items], pattern


def test_syntax_rules():
    for c in golden()["syntax"]:
        st = c["status"]
        if st == "ok":
            got = _interp_paths(c["pattern"], [c["subject"].encode("latin-1")])
            assert (int(got[0]) == 0) == c["match"], c
            continue
        with pytest.raises(L.L7Error) as e:
            L.RuleSet.compile_http([L.PortRuleHTTP(Path=c["pattern"])], dialect=RE2)
        want = {"invalid": [L.L7M_EINVAL_REGEX], "unsupported": [L.L7M_EUNSUPPORTED],
                "invalid_or_unsupported": [L.L7M_EINVAL_REGEX, L.L7M_EUNSUPPORTED]}[st]
        assert e.value.code in want, c


def test_search_differs_from_full_match():
    rules = [L.PortRuleHTTP(Path="/public/.*")]
    arena, offs = L.pack_http([L.HTTPRequest("GET", "/x/public/a", "h")])
    assert HttpProgram(L.RuleSet.compile_http(rules).program()).eval(arena, offs).tolist() == [-1]
    assert HttpProgram(L.RuleSet.compile_http(rules, dialect=RE2).program()).eval(arena, offs).tolist() == [0]


def test_multi_rule_first_match_vs_oracle():
    rng = np.random.default_rng(21)
    cases = golden()["search"]
    pats = sorted({c["pattern"] for c in cases})
    rules = []
    for i in range(60):
        rules.append(L.PortRuleHTTP(Path=str(rng.choice(pats)),
                                    Method=str(rng.choice(["", "GET", "^(GET|HEAD)$", "P"])),
                                    Host=str(rng.choice(["", "svc", "\\.local$"])),
                                    Headers=["x-t: v1"] if rng.random() < 0.2 else []))
    subjects = [c["subject"] for c in cases]
    reqs = [L.HTTPRequest(str(rng.choice(["GET", "POST", "HEAD", "PUT"])), str(rng.choice(subjects)),
                          str(rng.choice(["svc1.ns.local", "a.local", "example.com"])),
                          [("x-t", "v1")] if rng.random() < 0.5 else [])
            for _ in range(1500)]
    arena, offs = L.pack_http(reqs)
    got = HttpProgram(L.RuleSet.compile_http(rules, dialect=RE2).program()).eval(arena, offs)
    exp = HttpOracle(rules, dialect=RE2).eval(arena, offs)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]


def test_config2_1k_rules_compile_as_search_automata():
    """BASELINE config 2's 1000 rules compile under the RE2 dialect (search
    automata, program.h kDfaSearch: trailing repetitions cut, <= 32 patterns
    per automaton) and the program interpreter agrees with the oracle."""
    rules = W.rules(2)
    rs = L.RuleSet.compile_http(rules, dialect=RE2)
    prog = HttpProgram(rs.program())
    assert prog.h["search"] == 1
    kinds = [d["kind"] for d in prog.dfas[:prog.h["n_dfas"]]]
    # search automata (kind 1) and literal-anchored groups (kind 2: every
    # config-2 path pattern is /svc{i}/v... or /api/{w}/...: literal prefix L,
    # residual R shared by the group)
    assert kinds.count(1) + kinds.count(2) >= 1000 // 32
    assert kinds.count(2) >= 1000 // 32 and prog.fields[1][9] != 0xFFFFFFFF
    arena, offs = W.requests(2, 0, 1500)
    got = prog.eval(arena, offs)
    exp = HttpOracle(rules, dialect=RE2).eval(arena, offs, threads=8)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]


def test_search_trailing_repetition_cut_is_exact():
    """simplify_search: p X* / p X{n,m} at the end of a pattern match exactly
    where p / p X{n} do under search semantics; '$' after them keeps them."""
    cases = [("/a/.*", ["/a/", "x/a/", "/a", "/a/\nz"]), ("ab+", ["a", "ab", "xabbb"]),
             ("ab{2,4}", ["ab", "abb", "zabbbbbb"]), ("ab*$", ["a", "ab", "abx", "xabb"]),
             ("x*", ["", "y"]), ("(ab|cd)+", ["ab", "cdab", "ac"])]
    for pattern, subjects in cases:
        subs = [s.encode() for s in subjects]
        got = _interp_paths(pattern, subs)
        assert [int(v) == 0 for v in got] == [bool(regex_search(pattern, s)) for s in subs], pattern


def _gram_rules(rng, n):
    """Random RE2 path patterns, most with required literals (the gram filter's
    input) in every structural position: prefix, middle, repeated, inside
    groups, behind optional parts; some with none (always-walked groups)."""
    words = ["alpha", "bravo", "char", "delt", "echo1", "fox/", "/gol", "hot-", "ind.", "jul_"]
    out = []
    for i in range(n):
        w = str(rng.choice(words)) + str(i % 37)
        form = int(rng.integers(0, 9))
        p = ["/%s/v[0-9]+" % w, "[a-z]*%s(x|y)?" % w, "(%s)+z" % w, "^/(api|svc)/%s" % w, "%s{2}" % w,
             "q?%s[^/]*/" % w, "(ab|cd)[0-9]", "[a-c]{2,3}d", "%s$" % w][form]
        out.append(L.PortRuleHTTP(Path=p, Method=str(rng.choice(["", "GET", "(PUT|POST)"]))))
    return out


def _gram_subjects(rng, rules, n):
    """Paths that contain some rule's literal (hits and near misses)."""
    subs = []
    for _ in range(n):
        r = rules[int(rng.integers(0, len(rules)))].Path
        lit = "".join(ch for ch in r if ch.isalnum() or ch in "/-._")
        cut = int(rng.integers(0, len(lit) + 1))
        s = str(rng.choice(["", "/", "/api/", "/svc/", "xx"])) + lit[:cut] + str(rng.choice(["", "7", "z", "/", "v12/"]))
        if rng.random() < 0.3:
            s = s + s
        subs.append(s)
    return subs


def test_gram_filter_is_exact_on_random_literal_patterns():
    """program.h FieldDesc::gram_tab: with >= 3 search groups on :path the
    filter skips groups whose chosen grams a value lacks; the interpreter
    (walking only the selected groups, as the kernel does) equals the oracle,
    and the filter actually skips most groups."""
    rng = np.random.default_rng(33)
    for trial in range(3):
        rules = _gram_rules(rng, 200 + 100 * trial)
        prog = HttpProgram(L.RuleSet.compile_http(rules, dialect=RE2).program())
        fd = prog.fields[1]
        assert fd[4] != 0xFFFFFFFF, "path field without a gram filter"
        assert fd[9] != 0xFFFFFFFF, "path field without literal-anchored patterns"
        reqs = [L.HTTPRequest(str(rng.choice(["GET", "PUT", "POST"])), s) for s in _gram_subjects(rng, rules, 1500)]
        arena, offs = L.pack_http(reqs)
        got = prog.eval(arena, offs)
        exp = HttpOracle(rules, dialect=RE2).eval(arena, offs, threads=8)
        bad = np.nonzero(got != exp)[0]
        assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
        assert (exp >= 0).sum() > 100
        walked = [bin(prog.gram_select(1, r.path.encode())).count("1") for r in reqs[:300]]
        assert np.mean(walked) < 0.5 * fd[8]


def test_literal_anchored_patterns_exact():
    """program.h FieldDesc::alit_*: patterns L R (literal prefix L >= 4 bytes,
    residual R) are decided by gram probe + literal compare + the shared
    residual automaton.  Subjects repeat L, cut it, put it at the end, put a
    failing occurrence before a matching one, and R ends with '$' or is empty;
    the interpreter (the kernel's algorithm) equals the oracle (std::regex_search)."""
    rng = np.random.default_rng(44)
    lits = ["/svc%d/v" % i for i in range(40)] + ["/api/w%d/" % i for i in range(40)] + \
           ["abab%d" % i for i in range(20)] + ["aaaa", "aaab", "xyzw", "/a/b/c/d"]
    ress = ["", "[0-9]+/(users|items)/[0-9]", "x?$", "[a-c]*z", "(ab)+", "\\.json$", "[^/]+/.*"]
    pats = sorted({re_escape_lit(l) + str(rng.choice(ress)) for l in lits})
    rules = [L.PortRuleHTTP(Path=p) for p in pats]
    prog = HttpProgram(L.RuleSet.compile_http(rules, dialect=RE2).program())
    assert prog.fields[1][9] != 0xFFFFFFFF
    subs = []
    tails = ["", "12/users/7", "x", "zz", "ab", "abab", ".json", "q/r", "/", "9/items/0x"]
    for _ in range(3000):
        l1, l2 = str(rng.choice(lits)), str(rng.choice(lits))
        k = int(rng.integers(0, 6))
        if k == 0:
            s = l1 + str(rng.choice(tails))
        elif k == 1:
            s = l1[:-1] + str(rng.choice(tails))  # cut literal
        elif k == 2:
            s = l2 + "-" + l1 + str(rng.choice(tails))  # second occurrence decides
        elif k == 3:
            s = l1 + l1 + str(rng.choice(tails))  # overlapping / repeated
        elif k == 4:
            s = str(rng.choice(tails)) + l1  # literal at the end
        else:
            s = l1[:2] + l1 + str(rng.choice(tails))
        subs.append(s)
    arena, offs = L.pack_http([L.HTTPRequest("GET", s) for s in subs])
    got = prog.eval(arena, offs)
    exp = HttpOracle(rules, dialect=RE2).eval(arena, offs, threads=8)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(subs[i], int(exp[i]), int(got[i])) for i in bad[:10]]
    assert (exp >= 0).sum() > 600 and (exp == -1).sum() > 100


def re_escape_lit(s):
    return "".join("\\" + c if c in ".+*?()[]{}|^$\\" else c for c in s)


def test_alit_table_over_lds_budget_falls_back_to_search_groups():
    """a literal-anchored bucket table that does not fit the LDS
    budget used to fail the compile (L7M_ETOOBIG).  The field's patterns now
    fall back to search groups: every budget compiles, the small ones without
    the alit scan, and every program equals the oracle."""
    rules = W.rules(2, n_rules=300)
    arena, offs = W.requests(2, 0, 1200, n_rules=300)
    exp = HttpOracle(rules, dialect=RE2).eval(arena, offs, threads=8)
    seen = set()
    for budget in (1, 2048, 8192, 16384, 49152):
        prog = HttpProgram(L.RuleSet.compile_http(rules, dialect=RE2, lds_budget_bytes=budget).program())
        seen.add(prog.fields[1][9] != 0xFFFFFFFF)
        got = prog.eval(arena, offs)
        bad = np.nonzero(got != exp)[0]
        assert len(bad) == 0, (budget, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]])
    assert seen == {True, False}
