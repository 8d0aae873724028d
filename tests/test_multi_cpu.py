"""In-library multi-GPU (include/l7match.h l7m_multi_*): the C++ shard cuts
(l7m_shard_bounds) equal cilium_amd/dist.py's byte-balanced bounds, the
bench's process-per-GPU cut, on packed workloads; no GPU needed."""
import numpy as np
import pytest

from cilium_amd import dist as D
from cilium_amd import l7match as L
from cilium_amd import workloads as W


@pytest.mark.parametrize("cfg,n", [(2, 50_000), (3, 40_000), (5, 3_000), (1, 7)])
@pytest.mark.parametrize("parts", [1, 2, 3, 8])
def test_shard_bounds_equal_dist(cfg, n, parts):
    arena, offs = W.requests(cfg, 123_456, n, n_rules=200 if cfg != 1 else None)
    size = arena.nbytes - 64
    b = L.shard_bounds(offs, size, parts)
    exp = D.byte_balanced_bounds(offs, size, parts)
    assert [(int(b[k]), int(b[k + 1])) for k in range(parts)] == exp
    # equal bytes per shard to within one record
    bytes_ = [(int(offs[hi]) if hi < n else size) - (int(offs[lo]) if lo < n else size) for lo, hi in exp]
    assert max(bytes_) - min(bytes_) <= 2 * int(np.diff(offs).max()) if n > 1 else True


def test_shard_bounds_edges():
    assert L.shard_bounds(np.zeros(0, dtype=np.uint64), 0, 4).tolist() == [0, 0, 0, 0, 0]
    with pytest.raises(L.L7Error):
        L.shard_bounds(np.array([8, 0], dtype=np.uint64), 16, 2)  # not ascending
    with pytest.raises(L.L7Error):
        L.shard_bounds(np.array([0, 16], dtype=np.uint64), 16, 2)  # record past the arena


def test_device_set_needs_a_device():
    if L.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(L.L7Error):
        L.DeviceSet([0, 0])
