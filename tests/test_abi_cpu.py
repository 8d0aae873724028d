"""The plain C client (tests/cpp/abi_harness.c) links libl7match.so and,
without a HIP device, every l7m_eval fails loudly with L7M_EDEVICE (there is
no CPU evaluation path)."""
import pytest

from abi_files import run
from cilium_amd import l7match as L
from cilium_amd import workloads as W


def test_c_harness_links_and_fails_without_device(tmp_path):
    if L.device_count() > 0:
        pytest.skip("GPU present")
    rules = W.rules(2, n_rules=20)
    arena, offs = W.requests(2, 0, 64, n_rules=20)
    p, _ = run(str(tmp_path), rules, arena, offs, threads=2, iters=1)
    assert p.returncode == 1
    assert "l7m_eval -6" in p.stderr
