"""Zero-copy host path (l7m_api.cc mapped_host_range): l7m_eval on an arena in
pinned, device-mapped host memory runs the kernels on it in place (no H2D
staging copy).  Its verdicts and counters must equal the copying path's
(pageable arenas, or L7M_ZERO_COPY=0), which the oracle checks elsewhere;
misaligned arenas and ranges past the pinned allocation take the copying
path."""
import ctypes

import numpy as np
import pytest

from cilium_amd import l7match as L
from cilium_amd import workloads as W
import kafka_codec_cases as C
from oracle import HttpOracle, KafkaOracle

pytestmark = pytest.mark.gpu


class Pinned:
    def __init__(self, nbytes):
        self.p = ctypes.c_void_p()
        assert L._lib.l7m_alloc_pinned(nbytes, ctypes.byref(self.p)) == L.L7M_OK
        self.a = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self.p.value))

    def free(self):
        L._lib.l7m_free_pinned(self.p)


def _pinned_copy(arena, shift=0, slack=256):
    """The arena in pinned memory; the bytes around it (the 64-byte pad past
    arena_bytes included) are 0xff: the pad's contents must not matter."""
    pb = Pinned(arena.nbytes + shift + slack)
    pb.a[:] = 0xFF
    pb.a[shift:shift + arena.nbytes] = arena
    return pb, pb.a[shift:shift + arena.nbytes]


def _mapped(view):
    """Would l7m_eval read this arena in place? (l7m_api.cc: 16-byte aligned,
    and the padded range (arena_bytes + 64) & ~3 inside one pinned allocation)"""
    return bool(view.ctypes.data % 16 == 0 and L._lib.l7m_host_mapped(view.ctypes.data, (view.nbytes + 64) & ~3))


def _pinned_u64(x):
    pb = Pinned(x.nbytes + 64)
    v = pb.a[:x.nbytes].view(np.uint64)
    v[:] = x
    return pb, v


def test_http_zero_copy_matches_copying_path(gpu):
    rules = W.rules(2, n_rules=300)
    rs = L.RuleSet.compile_http(rules)
    arena, offs = W.requests(2, 0, 200_000, n_rules=300)
    hits_ref = np.zeros(rs.info.n_counters, dtype=np.uint64)
    ref = rs.eval(arena.copy(), offs, hits_ref)
    pa, view = _pinned_copy(arena)
    po, poffs = _pinned_u64(offs)
    try:
        assert _mapped(view), "the pinned arena must take the zero-copy path"
        assert L._lib.l7m_host_mapped(poffs.ctypes.data, poffs.nbytes) == 1
        for o in (offs, poffs):  # offsets copied, then read in place too
            hits = np.zeros_like(hits_ref)
            got = rs.eval(view, o, hits)
            assert np.array_equal(got, ref)
            assert np.array_equal(hits, hits_ref)
        exp = HttpOracle(rules).eval(arena, offs[:5000], threads=8)
        assert np.array_equal(ref[:5000], exp)
    finally:
        po.free()
        pa.free()


def test_http_zero_copy_falls_back_on_misaligned_or_short_ranges(gpu):
    rules = W.rules(2, n_rules=100)
    rs = L.RuleSet.compile_http(rules)
    arena, offs = W.requests(2, 0, 20_000, n_rules=100)
    ref = rs.eval(arena.copy(), offs)
    pa, view = _pinned_copy(arena, shift=4)  # arena pointer 4 mod 16: copying path
    # padded range past the allocation: an allocation of whole pages holding
    # the arena at its end, so the 64-byte pad cannot fit, whatever the
    # allocator rounds to
    size = (arena.nbytes + 15 + 4095) // 4096 * 4096
    pb = Pinned(size)
    at = (size - arena.nbytes) & ~15
    pb.a[at:at + arena.nbytes] = arena
    view2 = pb.a[at:at + arena.nbytes]
    try:
        assert not _mapped(view) and not _mapped(view2)
        assert np.array_equal(rs.eval(view, offs), ref)
        assert np.array_equal(rs.eval(view2, offs), ref)
    finally:
        pa.free()
        pb.free()


def test_kafka_zero_copy_with_compressed_sets(gpu):
    """Config-3 requests plus the compressed-set cases: the second pass
    (kafka_codec_kernel) also reads the arena in place."""
    rules = W.rules(3, n_rules=500)
    rs = L.RuleSet.compile_kafka(rules)
    arena, offs = W.requests(3, 0, 50_000, n_rules=500)
    ref = rs.eval(arena.copy(), offs)
    pa, view = _pinned_copy(arena)
    try:
        assert _mapped(view)
        assert np.array_equal(rs.eval(view, offs), ref)
    finally:
        pa.free()
    recs = [r for _, r, _ in C.request_cases()]
    carena, coffs = L.pack_records(recs)
    krs = L.RuleSet.compile_kafka([L.PortRuleKafka(Topic="t")])
    cref = krs.eval(carena.copy(), coffs)
    pc, cview = _pinned_copy(carena)
    try:
        assert np.array_equal(krs.eval(cview, coffs), cref)
    finally:
        pc.free()
    assert cref.tolist() == KafkaOracle([L.PortRuleKafka(Topic="t")]).eval(carena, coffs).tolist()
