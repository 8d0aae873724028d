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
