"""Reentrancy through the C ABI: 8 host threads of a plain C program
(tests/cpp/abi_harness.c, no ctypes) call l7m_eval concurrently on ONE
compiled handle; every thread's verdicts equal the oracle's and the summed
per-rule counters equal threads x iterations x one evaluation's."""
import numpy as np
import pytest

from abi_files import run
from cilium_amd import l7match as L
from cilium_amd import workloads as W
from oracle import HttpOracle

pytestmark = pytest.mark.gpu


def test_eight_threads_one_handle_c_harness(gpu, tmp_path):
    rules = W.rules(2)
    arena, offs = W.requests(2, 3_000_000, 50_000)
    threads, iters = 8, 3
    p, res = run(str(tmp_path), rules, arena, offs, threads, iters)
    assert p.returncode == 0, p.stderr[-2000:]
    verd, hits = res
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    assert np.array_equal(verd, exp)
    one = np.zeros(len(rules) + 2, dtype=np.uint64)
    L.RuleSet.compile_http(rules).eval(arena, offs, one)
    assert np.array_equal(hits, one * threads * iters)


def test_batcher_call_site_c_harness(gpu, tmp_path):
    """The call-site shape through the C ABI: 8 threads decide requests one
    at a time with the blocking l7m_batcher_eval (canAccess / decodeHeaders),
    a policy update (l7m_batcher_set_ruleset) lands halfway, denied requests
    get the 403 body; verdicts equal the oracle's, requests share batches,
    and the proxy stats add up."""
    rules = W.rules(2)
    arena, offs = W.requests(2, 5_000_000, 6_000)
    p, res = run(str(tmp_path), rules, arena, offs, 8, 1, batcher=True)
    assert p.returncode == 0, p.stderr[-2000:]
    verd, st = res
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    assert np.array_equal(verd, exp)
    batches, requests, denied, forwarded = (int(x) for x in st)
    assert requests == len(offs) and batches < requests // 4
    assert denied == int((exp == L.VERDICT_DENY).sum()) and forwarded == int((exp >= 0).sum())
