"""Config 5 on the GPU (BASELINE.json configs[4]):
adversarial path families ((a|aa)*b, .*(x|y).*(z|w).*q, 100-way literal
alternations, stacked [a-z]*, (.{0,8}){1,8}foo) at 10k and 100k rules, header
values of 1 KiB - 64 KiB (larger than the kernel's LDS stage, so they take
the HBM-direct path).

Oracle: the Thompson-NFA / Pike-VM simulator (oracle/nfa.h, engine "nfa"),
pinned against std::regex by tests/test_nfa_oracle_cpu.py.  std::regex
itself (the reference engine) backtracks exponentially on the `/f{i}/`
family's long tails and overflows its stack on long subjects (SURVEY.md
§0.8), so it checks only the small case here; every sample below is
compared unfiltered, including paths and values up to 64 KiB."""
import numpy as np
import pytest

from cilium_amd import l7match as L
from cilium_amd import workloads as W
import adversarial_cases as A
from oracle import HttpOracle

pytestmark = pytest.mark.gpu

_cache = {}


def compiled(n_rules):
    """(rules, product rule set, NFA oracle), compiled once per module."""
    if n_rules not in _cache:
        rules = W.rules(5, n_rules=n_rules)
        _cache[n_rules] = (rules, L.RuleSet.compile_http(rules), HttpOracle(rules, engine="nfa"))
    return _cache[n_rules]


def check(rs, orc, arena, offs, hits=True):
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    got = rs.eval(arena, offs, h if hits else None)
    exp = orc.eval(arena, offs, threads=16)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    if hits:
        assert int(h.sum()) == len(offs)
    return got


def test_adversarial_small_parity(gpu):
    """40 rules: the reference engine (std::regex) on the records it finishes,
    the NFA oracle on all of them."""
    rules = W.rules(5, n_rules=40)
    rs = L.RuleSet.compile_http(rules)
    arena, offs = W.requests(5, 0, 6000, n_rules=40)
    sizes = np.diff(np.append(offs.astype(np.int64), arena.nbytes - 64))
    assert sizes.max() > 32768  # some records exceed every LDS stage
    v = check(rs, HttpOracle(rules, engine="nfa"), arena, offs)
    assert (v >= 0).any() and (v == -1).any()
    a2, o2 = A.subset(arena, offs, A.cheap_for_oracle(arena, offs))
    check(rs, HttpOracle(rules), a2, o2)


@pytest.mark.parametrize("n_rules,n_req", [(10_000, 4000), (100_000, 1500)])
def test_adversarial_scale_parity(gpu, n_rules, n_req):
    """10k / 100k rules: one packed automaton per field (dfa_pack.h), the
    100k-rule path table walked from HBM/L2, global hit counters; every
    generated record, no filter."""
    rules, rs, orc = compiled(n_rules)
    assert rs.info.n_dfas == 4
    arena, offs = W.requests(5, 7_000_000, n_req, n_rules=n_rules)
    v = check(rs, orc, arena, offs)
    assert (v >= 0).sum() > len(v) // 4 and (v == -1).sum() > len(v) // 4
    # the records std::regex cannot finish are in the batch
    assert (~A.cheap_for_oracle(arena, offs)).sum() > n_req // 20


@pytest.mark.parametrize("n_rules", [10_000, 100_000])
def test_adversarial_long_fields_parity(gpu, n_rules):
    """Constructed paths and x-blob values up to 64 KiB (HBM-direct records):
    GPU == NFA oracle == the verdict the construction implies."""
    rules, rs, orc = compiled(n_rules)
    cases = A.long_field_cases(rules, 400, seed=n_rules) + A.blob_cases(rules, 120, seed=n_rules + 1)
    arena, offs = L.pack_http([c[0] for c in cases])
    exp = np.array([c[1] for c in cases], dtype=np.int32)
    got = check(rs, orc, arena, offs)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    assert max(len(c[0].path) for c in cases) > 60000


def test_adversarial_100k_full_batch_properties(gpu):
    """1M requests against 100k rules on the GPU: counters sum to N, a
    re-evaluation is identical, every allow names a rule whose /{family}{i}/
    prefix is the request's, and a strided sample of 4000 equals the NFA
    oracle."""
    rules, rs, orc = compiled(100_000)
    arena, offs = W.requests(5, 0, 1_000_000, n_rules=100_000, threads=16)
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    v = rs.eval(arena, offs, h)
    assert int(h.sum()) == len(offs)
    assert np.array_equal(rs.eval(arena, offs), v)
    assert set(np.unique(v[v < 0]).tolist()) <= {L.VERDICT_DENY}
    assert 0.3 < (v >= 0).mean() < 0.7
    keep = np.zeros(len(offs), dtype=bool)
    keep[::250] = True
    a2, o2 = A.subset(arena, offs, keep)
    exp = orc.eval(a2, o2, threads=16)
    bad = np.nonzero(v[keep] != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(v[keep][i])) for i in bad[:10]]
