"""Config 4 host side (no GPU): the mixed workload splits into a 5k-rule HTTP
part (config-2 generator) and a 5k-rule Kafka part (config-3 generator) under
seed 0xC4; both rule sets compile; per-protocol shards concatenate to the
unsharded stream (what bench.py's strong-scaling split relies on)."""
import numpy as np

from cilium_amd import dist as D
from cilium_amd import l7match as L
from cilium_amd import workloads as W


def test_mixed_parts_shape_and_compile():
    parts = W.mixed_parts(4)
    assert [(p[0], p[1], p[3]) for p in parts] == [(L.PROTO_HTTP, 2, 5000), (L.PROTO_KAFKA, 3, 5000)]
    assert sum(p[3] for p in parts) == W.CONFIGS[4]["n_rules"]
    for proto, gcfg, seed, n in parts:
        assert seed == 0xC4
        rules = W.rules(gcfg, seed=seed, n_rules=n)
        assert len(rules) == n
        rs = L.RuleSet.compile_http(rules) if proto == L.PROTO_HTTP else L.RuleSet.compile_kafka(rules)
        assert rs.n_counters == n + 2


def test_mixed_shards_concatenate():
    n_all, world = 1000, 4
    for proto, gcfg, seed, n in W.mixed_parts(4):
        whole, _ = W.requests(gcfg, 0, n_all, seed=seed, n_rules=n)
        chunks = []
        for r in range(world):
            lo, hi = D.shard_bounds(n_all, world, r)
            a, _ = W.requests(gcfg, lo, hi - lo, seed=seed, n_rules=n)
            chunks.append(a[:-64])
        assert np.array_equal(np.concatenate(chunks), whole[:-64])
