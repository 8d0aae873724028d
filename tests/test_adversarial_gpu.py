"""Config 5 on the GPU: adversarial patterns and records of up to 64 KiB
(larger than the kernel's LDS stage, so they take the HBM-direct path),
bit-exact against the oracle."""
import numpy as np
import pytest

from cilium_amd import workloads as W
from cilium_amd import l7match as L
from oracle import HttpOracle

pytestmark = pytest.mark.gpu
N_RULES = 40


def test_adversarial_parity(gpu):
    rules = W.rules(5, n_rules=N_RULES)
    arena, offs = W.requests(5, 0, 6000, n_rules=N_RULES)
    sizes = np.diff(np.append(offs.astype(np.int64), arena.nbytes - 64))
    assert sizes.max() > 32768  # some records exceed every LDS stage
    rs = L.RuleSet.compile_http(rules)
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    got = rs.eval(arena, offs, h)
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    assert int(h.sum()) == len(offs)


def test_adversarial_chunked_grouping_parity(gpu):
    # 66 path patterns: chunked grouping, 29 value DFAs whose end-code columns
    # take 116 KiB of LDS, so the compiler shrinks the LDS table image.
    rules = W.rules(5, n_rules=66)
    arena, offs = W.requests(5, 0, 3000, n_rules=66)
    rs = L.RuleSet.compile_http(rules)
    assert rs.info.n_dfas > 20
    got = rs.eval(arena, offs)
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]


def test_too_many_dfa_groups_fail_loudly(gpu):
    """More value DFAs than the kernel's LDS end-code columns hold (~30):
    l7m_eval returns L7M_ETOOBIG, no silent fallback."""
    rules = W.rules(5, n_rules=160)
    arena, offs = W.requests(5, 0, 100, n_rules=160)
    rs = L.RuleSet.compile_http(rules)
    with pytest.raises(L.L7Error) as e:
        rs.eval(arena, offs)
    assert e.value.code == L.L7M_ETOOBIG
