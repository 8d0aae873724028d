"""Config 5 on the GPU (BASELINE.json configs[4]):
adversarial path families ((a|aa)*b, .*(x|y).*(z|w).*q, 100-way literal
alternations, stacked [a-z]*, (.{0,8}){1,8}foo) at 10k and 100k rules, header
values of 1 KiB - 64 KiB (larger than the kernel's LDS stage, so they take
the HBM-direct path), bit-exact against the std::regex oracle.

Oracle cost: std::regex backtracks exponentially on `(.{0,8}){1,8}foo`
against long non-matching tails (seconds per request at 60 characters), so
the oracle-checked samples keep `/f{i}/` tails <= 24 bytes (the GPU verdicts of
the excluded records are covered by the size-independent checks)."""
import struct

import numpy as np
import pytest

from cilium_amd import workloads as W
from cilium_amd import l7match as L
from oracle import HttpOracle

pytestmark = pytest.mark.gpu


def cheap_for_oracle(arena, offs, max_f_tail=24):
    """Mask of records whose path the std::regex oracle evaluates quickly."""
    buf = arena.tobytes()
    keep = np.ones(len(offs), dtype=bool)
    for i, o in enumerate(offs.tolist()):
        w2, w3 = struct.unpack_from("<II", buf, o + 8)
        nh, ml, pl = w2 >> 24, w3 & 0xFFFF, w3 >> 16
        p = o + 20 + 4 * nh + ml
        path = buf[p:p + pl]
        if path.startswith(b"/f"):
            k = path.find(b"/", 1)
            keep[i] = k < 0 or pl - k - 1 <= max_f_tail
    return keep


def subset(arena, offs, keep):
    recs = []
    buf = arena.tobytes()
    for o in offs[keep].tolist():
        ln = struct.unpack_from("<I", buf, o)[0]
        recs.append(buf[o:o + ((ln + 3) & ~3)])
    return L.pack_records(recs)


def check(rules, arena, offs, rs=None, hits=True):
    rs = rs or L.RuleSet.compile_http(rules)
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    got = rs.eval(arena, offs, h if hits else None)
    exp = HttpOracle(rules).eval(arena, offs, threads=16)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    if hits:
        assert int(h.sum()) == len(offs)
    return got


def test_adversarial_small_parity(gpu):
    rules = W.rules(5, n_rules=40)
    arena, offs = W.requests(5, 0, 6000, n_rules=40)
    sizes = np.diff(np.append(offs.astype(np.int64), arena.nbytes - 64))
    assert sizes.max() > 32768  # some records exceed every LDS stage
    v = check(rules, arena, offs)
    assert (v >= 0).any() and (v == -1).any()


@pytest.mark.parametrize("n_rules,n_req", [(10_000, 3000), (100_000, 400)])
def test_adversarial_scale_parity(gpu, n_rules, n_req):
    """10k / 100k rules: one packed automaton per field (dfa_pack.h), the
    100k-rule path table walked from HBM/L2, global hit counters."""
    rules = W.rules(5, n_rules=n_rules)
    rs = L.RuleSet.compile_http(rules)
    assert rs.info.n_dfas == 4
    arena, offs = W.requests(5, 7_000_000, n_req, n_rules=n_rules)
    a2, o2 = subset(arena, offs, cheap_for_oracle(arena, offs))
    v = check(rules, a2, o2, rs)
    assert (v >= 0).sum() > len(v) // 4 and (v == -1).sum() > len(v) // 4


def test_adversarial_100k_full_batch_properties(gpu):
    """1M requests against 100k rules on the GPU: counters sum to N, every
    allow names a rule whose /{family}{i}/ prefix is the request's, and a
    re-evaluation is identical (the oracle cannot finish 1M here)."""
    rules = W.rules(5, n_rules=100_000)
    rs = L.RuleSet.compile_http(rules)
    arena, offs = W.requests(5, 0, 1_000_000, n_rules=100_000, threads=16)
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    v = rs.eval(arena, offs, h)
    assert int(h.sum()) == len(offs)
    assert np.array_equal(rs.eval(arena, offs), v)
    assert set(np.unique(v[v < 0]).tolist()) <= {L.VERDICT_DENY}
    assert 0.3 < (v >= 0).mean() < 0.7
    buf = arena.tobytes()
    idx = np.nonzero(v >= 0)[0][:: 997]
    for i in idx.tolist():
        o = int(offs[i])
        w2, w3 = struct.unpack_from("<II", buf, o + 8)
        p = o + 20 + 4 * (w2 >> 24) + (w3 & 0xFFFF)
        path = buf[p:p + (w3 >> 16)]
        fam = rules[int(v[i])].Path.split("/")[1]
        assert path.startswith(("/" + fam + "/").encode()), (path[:20], fam)
