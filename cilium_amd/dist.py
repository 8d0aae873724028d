"""Multi-GPU plumbing of the batched verdict path.

Requests are independent, so a batch shards across ranks with no data-path
collective: one process per GPU, each evaluating a contiguous range of
records against a replicated compiled rule set.  The only collective is the
sum of the per-rule hit / deny counters ([0] denies, [1] parse errors,
[2 + i] allowed by rule i), an all-reduce of R + 2 uint64 over RCCL (backend
"nccl") on GPUs, or gloo on CPU.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Equal-count contiguous shard [start, end) of n records for `rank`."""
    return n * rank // world, n * (rank + 1) // world


def byte_balanced_bounds(offsets: np.ndarray, arena_bytes: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous record ranges whose arena bytes are as equal as possible
    (HBM traffic per GPU is what has to balance).  offsets: ascending uint64."""
    n = int(offsets.shape[0])
    if n == 0:
        return [(0, 0)] * world
    starts = offsets.astype(np.int64)
    first = int(starts[0])
    total = int(arena_bytes) - first
    cuts = [0]
    for r in range(1, world):
        target = first + total * r // world
        cuts.append(int(np.searchsorted(starts, target, side="left")))
    cuts.append(n)
    for i in range(1, len(cuts)):
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


def cuts_from_block_bytes(block_bytes: np.ndarray, block: int, n: int, world: int) -> List[Tuple[int, int]]:
    """Byte-balanced contiguous shards of n records from per-block byte sums:
    the cut for rank r lies where the cumulative bytes reach r / world of the
    total, interpolated inside its block (equal HBM traffic
    per GPU)."""
    if n == 0:
        return [(0, 0)] * world
    bb = np.asarray(block_bytes, dtype=np.float64)
    cum = np.cumsum(bb)
    total = float(cum[-1]) if cum.size else 0.0
    cuts = [0]
    for r in range(1, world):
        if not total:
            cuts.append(n * r // world)
            continue
        target = total * r / world
        j = int(np.searchsorted(cum, target, side="left"))  # the block holding the target byte
        before = float(cum[j - 1]) if j else 0.0
        in_blk = min(block, n - j * block)
        frac = (target - before) / bb[j] if bb[j] else 0.0
        cuts.append(min(n, j * block + int(round(frac * in_blk))))
    cuts.append(n)
    for i in range(1, len(cuts)):
        cuts[i] = min(n, max(cuts[i], cuts[i - 1]))
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


def balanced_shard(config: int, n: int, world: int, rank: int, block: int = 1 << 16, threads: int = 8,
                   seed=None, n_rules=None, device=None) -> Tuple[int, int]:
    """This rank's byte-balanced range of a deterministic workload of n
    requests (cilium_amd/workloads.py).  Each rank sizes an equal share of the
    blocks (sizes only, no records written), the per-block byte sums are
    all-gathered (one collective at setup, outside the timed region), and all
    ranks cut the same bounds."""
    from . import workloads as W
    nb = (n + block - 1) // block
    b0, b1 = nb * rank // world, nb * (rank + 1) // world
    lo, hi = b0 * block, min(n, b1 * block)
    mine = W.block_bytes(config, lo, max(0, hi - lo), block, seed=seed, n_rules=n_rules, threads=threads)
    if world > 1:
        import torch
        import torch.distributed as dist
        dev = device if device is not None else torch.device("cpu")
        t = torch.zeros(nb, dtype=torch.float64, device=dev)
        t[b0:b1] = torch.from_numpy(mine.astype(np.float64)).to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        allb = t.cpu().numpy()
    else:
        allb = mine.astype(np.float64)
    return cuts_from_block_bytes(allb, block, n, world)[rank]


def counters_from_verdicts(verdicts: np.ndarray, n_rules: int) -> np.ndarray:
    """Host statement of the kernels' counter semantics (include/l7match.h):
    [0] denies, [1] parse errors + unsupported, [2 + i] allowed by rule i;
    L7M_VERDICT_ALLOW_NO_L7 is not counted."""
    v = np.asarray(verdicts, dtype=np.int64)
    out = np.zeros(n_rules + 2, dtype=np.uint64)
    out[0] = np.count_nonzero(v == -1)
    out[1] = np.count_nonzero(v <= -2)
    allowed = v[(v >= 0) & (v < n_rules)]
    if allowed.size:
        out[2:] += np.bincount(allowed, minlength=n_rules).astype(np.uint64)
    return out


def allreduce_counters(t, group=None):
    """Sum per-rank counters in place (torch tensor, int64 / uint64 bits)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t
