"""Config 4 on the GPU: the 5k-rule HTTP and 5k-rule Kafka parts of the mixed
workload (W.mixed_parts), each evaluated through the C ABI on its own HIP
stream concurrently, bit-exact against the oracle; counters of both parts
concatenated as bench.py all-reduces them."""
import numpy as np
import pytest
import torch

from cilium_amd import workloads as W
from cilium_amd import l7match as L
from oracle import HttpOracle, KafkaOracle

pytestmark = pytest.mark.gpu
N_REQ = 3000


def test_mixed_parts_concurrent_streams(gpu):
    dev = torch.device("cuda", 0)
    parts = []
    for proto, gcfg, seed, n_rules in W.mixed_parts(4):
        rules = W.rules(gcfg, seed=seed, n_rules=n_rules)
        rs = L.RuleSet.compile_http(rules) if proto == L.PROTO_HTTP else L.RuleSet.compile_kafka(rules)
        arena, offs = W.requests(gcfg, 5_000_000, N_REQ, seed=seed, n_rules=n_rules)
        orc = HttpOracle(rules) if proto == L.PROTO_HTTP else KafkaOracle(rules)
        parts.append((rs, arena, offs, orc.eval(arena, offs, threads=8)))
    n_cnt = [p[0].n_counters for p in parts]
    d_hits = torch.zeros(sum(n_cnt), dtype=torch.int64, device=dev)
    views = [d_hits[:n_cnt[0]], d_hits[n_cnt[0]:]]
    outs, streams = [], []
    for (rs, arena, offs, _), hv in zip(parts, views):
        s = torch.cuda.Stream(device=dev)
        d_arena = torch.from_numpy(arena).to(dev)
        d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_verd = torch.full((len(offs),), -7, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        rs.eval_device(d_arena, arena.nbytes, d_offs, len(offs), d_verd, hv, s.cuda_stream, 0)
        outs.append((d_arena, d_offs, d_verd))
        streams.append(s)
    torch.cuda.synchronize()
    for (rs, arena, offs, exp), (_, _, d_verd), hv in zip(parts, outs, views):
        got = d_verd.cpu().numpy()
        bad = np.nonzero(got != exp)[0]
        assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
        h = hv.cpu().numpy()
        assert int(h.sum()) == len(offs)
        # counters: [0] deny, [1] parse error / unsupported, [2+i] first allowing rule i
        assert int(h[0]) == int((exp == -1).sum())
        allowed = exp[exp >= 0]
        assert np.array_equal(h[2:], np.bincount(allowed, minlength=len(h) - 2)[: len(h) - 2])
