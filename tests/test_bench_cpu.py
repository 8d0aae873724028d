"""bench.py's parity leg (the oracle sample of the timed batch's verdicts),
exercised on CPU with verdicts the oracle itself produced."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from cilium_amd import workloads as W  # noqa: E402
from oracle import HttpOracle, KafkaOracle  # noqa: E402


def _verdicts(cfg, lo, n, rules):
    a, o = W.requests(cfg, lo, n, n_rules=len(rules))
    orc = HttpOracle(rules) if cfg != 3 else KafkaOracle(rules)
    return orc.eval(a, o, threads=4)


def test_parity_leg_http_strided_sample_and_mismatch():
    rules = W.rules(2)
    lo, n = 123_456, 20_000
    v = _verdicts(2, lo, n, rules)
    r = bench.parity_leg(2, rules, v, lo, n, threads=4, n_sample=3000, blocks=16)
    assert r["mismatches"] == 0 and r["runs"] == 16 and r["sampled"] == 16 * 188
    bad = v.copy()
    bad[n - 1] = -7  # the last run ends at the shard's last request
    r = bench.parity_leg(2, rules, bad, lo, n, threads=4, n_sample=3000, blocks=16)
    assert r["mismatches"] == 1 and r["first_mismatch"] == {"request": lo + n - 1, "gpu": -7,
                                                            "oracle": int(v[n - 1])}


def test_parity_leg_kafka_whole_small_shard():
    rules = W.rules(3, n_rules=500)
    v = _verdicts(3, 0, 1000, rules)
    r = bench.parity_leg(3, rules, v, 0, 1000, threads=4, n_sample=5000, n_rules=500)
    assert r == {**r, "sampled": 1000, "mismatches": 0, "runs": 1}
