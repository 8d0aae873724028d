"""In-library multi-GPU (include/l7match.h l7m_multi_*) on
the GPU box's card: a device set that names device 0 twice runs two
byte-balanced shards concurrently on two streams; verdicts and counters must
equal one l7m_eval over the whole batch bit for bit (HTTP config 2, Kafka
config 3 with an L7DataMap, device-resident shards).  RCCL needs distinct
devices, so this set sums its counters on the host; the RCCL all-reduce
runs on a node with several GPUs (uses_rccl)."""
import numpy as np
import pytest
import torch

from cilium_amd import l7match as L
from cilium_amd import workloads as W

pytestmark = pytest.mark.gpu


def _ref(rs, arena, offs, ids=None):
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    v = rs.eval(arena, offs, h) if ids is None else rs.eval(arena, offs, h, identities=ids)
    return v, h


@pytest.mark.parametrize("devs", [[0], [0, 0], [0, 0, 0]])
def test_device_set_http_equals_one_eval(gpu, devs):
    rules = W.rules(2)
    rs = L.RuleSet.compile_http(rules)
    arena, offs = W.requests(2, 7_000_000, 300_000)
    exp, eh = _ref(rs, arena, offs)
    ds = L.DeviceSet(devs)
    assert not ds.uses_rccl
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    got = ds.eval(rs, arena, offs, h)
    assert np.array_equal(got, exp)
    assert np.array_equal(h, eh)
    h2 = h.copy()
    ds.eval(rs, arena, offs, h2)  # counters accumulate
    assert np.array_equal(h2, 2 * eh)
    ds.close()


def test_device_set_kafka_map_and_device_shards(gpu):
    import selector_cases as S
    entries, idmap = S.random_map(23, n_rules=600, n_ids=12)
    rs = L.RuleSet.compile_kafka_map(entries, idmap)
    arena, offs = W.requests(3, 9_000_000, 120_000, n_rules=600)
    ids = S.request_identities(29, len(offs), idmap)
    exp, eh = _ref(rs, arena, offs, ids)
    ds = L.DeviceSet([0, 0])
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    assert np.array_equal(ds.eval(rs, arena, offs, h, identities=ids), exp)
    assert np.array_equal(h, eh)
    # device-resident shards cut by l7m_shard_bounds
    size = arena.nbytes - 64
    b = L.shard_bounds(offs, size, 2)
    shards, keep = [], []
    for k in range(2):
        lo, hi = int(b[k]), int(b[k + 1])
        a0 = int(offs[lo])
        a1 = int(offs[hi]) if hi < len(offs) else size
        da = torch.zeros(((a1 - a0 + 64 + 15) // 16) * 16, dtype=torch.uint8, device="cuda:0")
        da[:a1 - a0] = torch.from_numpy(arena[a0:a1].copy()).cuda()
        do = torch.from_numpy((offs[lo:hi] - np.uint64(a0)).view(np.int64)).cuda()
        di = torch.from_numpy(ids[lo:hi].view(np.int32)).cuda()
        dv = torch.empty(hi - lo, dtype=torch.int32, device="cuda:0")
        keep.append(dv)
        shards.append((da, a1 - a0, do, hi - lo, dv, di))
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    torch.cuda.synchronize()  # the set's own streams are not ordered after torch's (include/l7match.h)
    ds.eval_device(rs, shards, h)
    got = torch.cat(keep).cpu().numpy()
    assert np.array_equal(got, exp)
    assert np.array_equal(h, eh)
    ds.close()
