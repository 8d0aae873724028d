"""Config 5: NFA-heavy path families ((a|aa)*b, wildcards,
100-way alternations, stacked [a-z]*, (.{0,8}){1,8}foo) and header values of
1 KiB - 64 KiB, compiler checked through the program interpreter against the
oracle.  Oracle limits: std::regex backtracks, so generated subjects keep
(a|aa)* runs <= 20 characters; the long values are literal-compared."""
import numpy as np

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


def test_adversarial_chunked_grouping_vs_oracle():
    """> 64 path patterns that do not fit one DFA group: estimate-based
    chunking (http_compile.cc build_groups) then halving; verdicts unchanged."""
    rules = W.rules(5, n_rules=160)
    arena, offs = W.requests(5, 0, 50, n_rules=160)
    rs = L.RuleSet.compile_http(rules)
    assert rs.info.n_dfas > 10
    got = HttpProgram(rs.program()).eval(arena, offs)
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
