"""Multi-process (world_size 2, gloo, CPU) tests of the sharded path: each rank
evaluates its contiguous shard of the same deterministic workload and the
per-rule counters are summed with an all-reduce; the result must equal the
single-process counters.  The verdict computation here is the CPU oracle (the
checker) because this container has no GPU; the GPU path is the same plumbing
around l7m_eval_device (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cilium_amd import dist as D
from cilium_amd import workloads as W

N = 6000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cfg, n_rules, out_dir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    from oracle import HttpOracle, KafkaOracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rules = W.rules(cfg, n_rules=n_rules)
    # byte-balanced shard: block byte sums all-reduced over gloo (bench.py's path)
    start, end = D.balanced_shard(cfg, N, world, rank, block=512, threads=1, n_rules=n_rules)
    np.save(os.path.join(out_dir, f"b{rank}.npy"), np.array([start, end]))
    arena, offs = W.requests(cfg, start, end - start, n_rules=n_rules, threads=1)
    orc = HttpOracle(rules) if cfg != 3 else KafkaOracle(rules)
    v = orc.eval(arena, offs)
    ctr = torch.from_numpy(D.counters_from_verdicts(v, len(rules)).view(np.int64).copy())
    D.allreduce_counters(ctr)
    np.save(os.path.join(out_dir, f"ctr{rank}.npy"), ctr.numpy())
    np.save(os.path.join(out_dir, f"v{rank}.npy"), v)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg,n_rules", [(2, 300), (3, 2000)])
def test_two_rank_sharded_counters_equal_single_process(tmp_path, cfg, n_rules):
    from oracle import HttpOracle, KafkaOracle
    mp.start_processes(_worker, args=(2, _free_port(), cfg, n_rules, str(tmp_path)), nprocs=2,
                       start_method="spawn", join=True)
    rules = W.rules(cfg, n_rules=n_rules)
    arena, offs = W.requests(cfg, 0, N, n_rules=n_rules)
    orc = HttpOracle(rules) if cfg != 3 else KafkaOracle(rules)
    v = orc.eval(arena, offs)
    full = D.counters_from_verdicts(v, len(rules)).view(np.int64)
    for r in range(2):
        assert (np.load(tmp_path / f"ctr{r}.npy") == full).all()
    shards = np.concatenate([np.load(tmp_path / f"v{r}.npy") for r in range(2)])
    assert (shards == v).all()  # shard invariance of the deterministic workload
    b0, b1 = np.load(tmp_path / "b0.npy"), np.load(tmp_path / "b1.npy")
    assert b0[0] == 0 and b0[1] == b1[0] and b1[1] == N
    nbytes = arena.nbytes - 64
    halves = [int(offs[b0[1]]), nbytes - int(offs[b0[1]])]
    assert abs(halves[0] - halves[1]) < 0.01 * nbytes  # equal HBM bytes per rank


def test_byte_balanced_bounds_cover_and_balance():
    arena, offs = W.requests(2, 0, 20000, n_rules=200)
    nbytes = arena.nbytes - 64
    for world in (1, 2, 4, 8):
        b = D.byte_balanced_bounds(offs, nbytes, world)
        assert b[0][0] == 0 and b[-1][1] == len(offs)
        assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
        sizes = [(int(offs[e]) if e < len(offs) else nbytes) - int(offs[s]) for s, e in b]
        assert max(sizes) - min(sizes) <= 2 * 1024


def test_block_byte_cuts_match_exact_byte_balance():
    """dist.cuts_from_block_bytes (bench.py: block sums, interpolated) lands
    within one block's imbalance of the exact per-record split."""
    n = 50_000
    arena, offs = W.requests(2, 0, n, n_rules=300)
    nbytes = arena.nbytes - 64
    for block in (256, 4096):
        bb = W.block_bytes(2, 0, n, block, n_rules=300)
        assert int(bb.sum()) == nbytes
        for world in (2, 3, 8):
            cuts = D.cuts_from_block_bytes(bb, block, n, world)
            assert cuts[0][0] == 0 and cuts[-1][1] == n
            assert all(cuts[i][1] == cuts[i + 1][0] for i in range(world - 1))
            sizes = [(int(offs[e]) if e < n else nbytes) - int(offs[s]) for s, e in cuts]
            assert max(sizes) - min(sizes) <= 0.02 * nbytes / world + 2048, (block, world, sizes)


def test_counters_from_verdicts_semantics():
    v = np.array([-1, -2, -3, 0, 2, 2, 0x7FFFFFFF], dtype=np.int32)
    c = D.counters_from_verdicts(v, 3)
    assert c.tolist() == [1, 2, 1, 0, 2]
    assert D.shard_bounds(10, 3, 0) == (0, 3) and D.shard_bounds(10, 3, 2) == (6, 10)


def _mixed_worker(rank, world, port, n_all, out_dir):
    """Config 4 as bench.run_mixed does it: per protocol part, this rank's
    1/world of the part's requests; counters of both parts concatenated into
    ONE buffer, one all-reduce."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    from oracle import HttpOracle, KafkaOracle
    from cilium_amd import l7match as L

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctrs = []
    for proto, gcfg, seed, n_rules in W.mixed_parts(4):
        rules = W.rules(gcfg, seed=seed, n_rules=n_rules)
        lo, hi = D.shard_bounds(n_all, world, rank)
        arena, offs = W.requests(gcfg, lo, hi - lo, seed=seed, n_rules=n_rules, threads=1)
        orc = HttpOracle(rules) if proto == L.PROTO_HTTP else KafkaOracle(rules)
        ctrs.append(D.counters_from_verdicts(orc.eval(arena, offs), len(rules)).view(np.int64))
    ctr = torch.from_numpy(np.concatenate(ctrs))
    D.allreduce_counters(ctr)
    np.save(os.path.join(out_dir, f"mixed{rank}.npy"), ctr.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_mixed_config4_counters(tmp_path):
    from oracle import HttpOracle, KafkaOracle
    from cilium_amd import l7match as L
    n_all = 800
    mp.start_processes(_mixed_worker, args=(2, _free_port(), n_all, str(tmp_path)), nprocs=2,
                       start_method="spawn", join=True)
    full = []
    for proto, gcfg, seed, n_rules in W.mixed_parts(4):
        rules = W.rules(gcfg, seed=seed, n_rules=n_rules)
        arena, offs = W.requests(gcfg, 0, n_all, seed=seed, n_rules=n_rules)
        orc = HttpOracle(rules) if proto == L.PROTO_HTTP else KafkaOracle(rules)
        full.append(D.counters_from_verdicts(orc.eval(arena, offs), len(rules)).view(np.int64))
    full = np.concatenate(full)
    assert int(full.sum()) == 2 * n_all
    for r in range(2):
        assert (np.load(tmp_path / f"mixed{r}.npy") == full).all()
