"""Config 5: NFA-heavy path families ((a|aa)*b, wildcards,
100-way alternations, stacked [a-z]*, (.{0,8}){1,8}foo) and header values of
1 KiB - 64 KiB, compiler checked through the program interpreter against the
oracle.  Oracle limits: std::regex backtracks, so generated subjects keep
(a|aa)* runs <= 20 characters; the long values are literal-compared."""
import numpy as np
import pytest

from cilium_amd import workloads as W
from cilium_amd import l7match as L
from oracle import HttpOracle
from program_interp import HttpProgram

N_RULES = 40


def test_adversarial_compiler_vs_oracle():
    rules = W.rules(5, n_rules=N_RULES)
    arena, offs = W.requests(5, 0, 200, n_rules=N_RULES)
    rs = L.RuleSet.compile_http(rules)
    got = HttpProgram(rs.program()).eval(arena, offs)
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    assert (exp >= 0).any() and (exp == -1).any()


def test_adversarial_scale_one_automaton_per_field():
    """2k adversarial rules compile into ONE packed automaton per field
    (literal-prefix product + shared residual tails, dfa_pack.h) in seconds,
    and the packed program agrees with the oracle."""
    import time
    rules = W.rules(5, n_rules=2000)
    t = time.time()
    rs = L.RuleSet.compile_http(rules)
    assert time.time() - t < 60
    # method, path, x-blob value + the header-name automaton
    assert rs.info.n_dfas == 4
    arena, offs = W.requests(5, 0, 120, n_rules=2000)
    got = HttpProgram(rs.program()).eval(arena, offs)
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    assert (exp >= 0).any() and (exp == -1).any()


def test_many_dfa_groups_are_rejected_at_compile_time():
    """A rule set whose fixed LDS part (per-lane end-code columns of every
    value DFA group) cannot fit the kernel is refused by l7m_compile_http,
    where Envoy would NACK the policy, not on every batch."""
    rules = [L.PortRuleHTTP(Path=f".*x{i}y.*") for i in range(400)]
    with pytest.raises(L.L7Error) as e:  # a tiny product-state limit splits the set into ~400 groups
        L.RuleSet.compile_http(rules, max_dfa_states=8)
    assert e.value.code == L.L7M_ETOOBIG
    assert "fixed LDS" in str(e.value)


def test_literal_tables_of_hbm_walked_dfas():
    """Config 5's x-blob literals (1 KiB header values) sit in HBM-walked
    automata: their DFAs carry literal tables (program.h DfaDesc::lit_tab)
    whose entries hold exactly the rules' values, so the kernel can compare a
    latched literal directly (l7m_kernels.hip walk_hbm)."""
    import numpy as np
    from program_interp import HttpProgram, KNONE
    rules = W.rules(5, n_rules=2000)
    blobs = {h.split(": ", 1)[1] for r in rules for h in r.Headers if h.lower().startswith("x-blob")}
    assert blobs
    rs = L.RuleSet.compile_http(rules)
    prog = rs.program()
    P = HttpProgram(prog)
    raw = prog.astype(np.uint32).tobytes()
    found = set()
    for d in P.dfas[:P.h["n_dfas"]]:
        if d["lit_tab"] == KNONE:
            continue
        assert d["lds_table"] == KNONE  # only HBM-walked automata carry them
        for p in range(d["npats"]):
            off, n = P.w[d["lit_tab"] + 2 * p], P.w[d["lit_tab"] + 2 * p + 1]
            if off != KNONE:
                found.add(raw[4 * off: 4 * off + n].decode())
    assert found == {b for b in blobs if len(b) >= 16}
