"""World-size-2 sharded path with the PRODUCT kernels: two processes (gloo
for the counter all-reduce, both on cuda:0 of the one-GPU box) each evaluate
their contiguous shard with l7m_eval_device on HBM-resident buffers; the
concatenated verdicts equal the oracle's and the all-reduced kernel counters
equal the single-process kernel counters.  bench.py --gpus N runs the same
plumbing over RCCL with one GPU per rank (multi-GPU scaling itself is
measured only by the driver's 8-GPU runs)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cilium_amd import dist as D
from cilium_amd import workloads as W

pytestmark = pytest.mark.gpu
N = 200_000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cfg, n_rules, out_dir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    from cilium_amd import l7match as L

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    rules = W.rules(cfg, n_rules=n_rules)
    rs = L.RuleSet.compile_http(rules) if cfg != 3 else L.RuleSet.compile_kafka(rules)
    start, end = D.shard_bounds(N, world, rank)
    arena, offs = W.requests(cfg, start, end - start, n_rules=n_rules, threads=4)
    d_arena = torch.from_numpy(arena).cuda()
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    d_v = torch.empty(end - start, dtype=torch.int32, device="cuda")
    d_h = torch.zeros(rs.n_counters, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    rs.eval_device(d_arena, arena.nbytes, d_offs, end - start, d_v, d_h, s.cuda_stream)
    torch.cuda.synchronize()
    ctr = d_h.cpu()
    D.allreduce_counters(ctr)  # gloo here; RCCL in bench.py
    np.save(os.path.join(out_dir, f"ctr{rank}.npy"), ctr.numpy())
    np.save(os.path.join(out_dir, f"v{rank}.npy"), d_v.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg,n_rules", [(2, 1000), (3, 10000)])
def test_two_rank_product_shards_equal_single_process(gpu, tmp_path, cfg, n_rules):
    from cilium_amd import l7match as L
    from oracle import HttpOracle, KafkaOracle
    mp.start_processes(_worker, args=(2, _free_port(), cfg, n_rules, str(tmp_path)), nprocs=2,
                       start_method="spawn", join=True)
    rules = W.rules(cfg, n_rules=n_rules)
    arena, offs = W.requests(cfg, 0, N, n_rules=n_rules, threads=8)
    rs = L.RuleSet.compile_http(rules) if cfg != 3 else L.RuleSet.compile_kafka(rules)
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    v_single = rs.eval(arena, offs, h)
    v = np.concatenate([np.load(tmp_path / f"v{r}.npy") for r in range(2)])
    assert np.array_equal(v, v_single)
    orc = HttpOracle(rules) if cfg != 3 else KafkaOracle(rules)
    assert np.array_equal(v, orc.eval(arena, offs, threads=8))
    for r in range(2):
        assert np.array_equal(np.load(tmp_path / f"ctr{r}.npy").view(np.uint64), h)
    assert np.array_equal(h, D.counters_from_verdicts(v, len(rules)))
