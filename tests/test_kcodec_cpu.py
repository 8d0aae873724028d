"""Compressed Kafka message sets on the CPU: the oracle (zlib + restated Go
gzip framing, restated golang/snappy) against the reference semantics case by
case, and the GPU second pass's decoder (cilium_amd/csrc/l7m_kcodec.h, built
for the host as tests/cpp/bin/libkcodec.so) against the oracle on every case
and on thousands of random corruptions of valid gzip / snappy values."""
import ctypes
import os
import random

import numpy as np
import pytest

import kafka_codec_cases as C
import kafka_wire as K
from cilium_amd import l7match as L
from oracle import KafkaOracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SLAB = 2 * 100 * 65535 + 65536  # the product's slab (l7m_api.cc)


def _kcodec():
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "cpp", "bin", "libkcodec.so"))
    lib.kc_host_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint32]
    lib.kc_host_check_produce.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32]
    return lib


def _oracle(records, topic="t"):
    arena, offs = L.pack_records(records)
    return KafkaOracle([L.PortRuleKafka(Topic=topic)]).eval(arena, offs).tolist()


@pytest.mark.parametrize("case", C.request_cases(), ids=lambda c: c[0])
def test_oracle_compressed_sets_follow_reference(case):
    name, rec, exp = case
    assert _oracle([rec]) == [exp], name


def test_oracle_compressed_deny_cases():
    for name, rec, exp in C.deny_cases():
        assert _oracle([rec], topic="x") == [exp], name


def test_device_decoder_matches_oracle_on_cases():
    lib = _kcodec()
    for name, codec, val, ver, exp in C.value_cases():
        rc = lib.kc_host_check(val, len(val), codec, ver, SLAB)
        assert rc == (0 if exp == 0 else 1), (name, rc)


def test_device_decoder_matches_oracle_on_random_corruptions():
    lib = _kcodec()
    rnd = random.Random(7)
    base = [(K.GZIP, K.gzip_member(C.INNER)), (K.GZIP, K.gzip_member(C.INNER, level=1)),
            (K.GZIP, K.gzip_member(C.INNER, strategy=3)), (K.SNAPPY, K.snappy_block(C.INNER)),
            (K.SNAPPY, K.snappy_java(C.INNER, chunk=40)), (K.GZIP, K.gzip_member(C.INNER, level=0))]
    recs, got = [], []
    for _ in range(3000):
        codec, v = rnd.choice(base)
        v = bytearray(v)
        for _ in range(rnd.randrange(1, 4)):
            k = rnd.randrange(4)
            if k == 0 and v:
                v[rnd.randrange(len(v))] ^= 1 << rnd.randrange(8)
            elif k == 1 and v:
                v[rnd.randrange(len(v))] = rnd.randrange(256)
            elif k == 2 and len(v) > 1:
                del v[rnd.randrange(len(v)):]
            else:
                v += bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 12)))
        v = bytes(v)
        got.append(lib.kc_host_check(v, len(v), codec, 1, SLAB))
        recs.append(K.produce(1, "c", [("t", [(0, K.wrapper_set(v, codec, 1))])]))
    exp = _oracle(recs)
    mism = [(i, exp[i], got[i]) for i in range(len(recs)) if (exp[i] == 0) != (got[i] == 0) or exp[i] not in (0, -2)]
    assert not mism, mism[:10]
    assert 0 < sum(1 for e in exp if e == 0) < len(exp)  # both outcomes exercised


def test_device_decoder_nesting_and_slab_limits():
    lib = _kcodec()
    ok8 = C.deep_nesting(8)
    assert _oracle([ok8, C.deep_nesting(9)]) == [0, 0]
    # values of deep_nesting(n): the decoder follows 8 levels, reports 9 as unsupported
    for n, want in ((8, 0), (9, 2)):
        v = K.gzip_member(C.INNER)
        for _ in range(n - 1):
            v = K.gzip_member(K.wrapper_set(v, K.GZIP, 1))
        assert lib.kc_host_check(v, len(v), K.GZIP, 1, SLAB) == want
    # a slab too small for a decoded set below maxParseBufSize: unsupported, not an error
    big = K.gzip_member(K.message_set(["x" * 300_000], version=1))
    assert lib.kc_host_check(big, len(big), K.GZIP, 1, 100_000) == 2
    assert lib.kc_host_check(big, len(big), K.GZIP, 1, SLAB) == 0


def test_second_pass_request_walk_matches_oracle_on_cases():
    """kc_check_produce (the GPU second pass per queued request) on every
    request case: a ReadRequest error exactly where the oracle has -2."""
    lib = _kcodec()
    for name, rec, exp in C.request_cases():
        rc = lib.kc_host_check_produce(rec, len(rec), SLAB)
        assert rc in (0, 1) and (rc == 1) == (exp == -2), (name, rc, exp)


def test_second_pass_request_walk_matches_oracle_on_random_requests():
    """Multi-topic / multi-partition produce requests mixing plain and
    compressed messages, a third of the compressed values corrupted: the
    second pass re-walks every set and fails exactly the requests the
    oracle fails (the first pass accepts all of them: framing is valid)."""
    lib = _kcodec()
    recs = C.random_produce_requests(random.Random(5), 1500)
    exp = _oracle(recs)
    got = [lib.kc_host_check_produce(r, len(r), SLAB) for r in recs]
    mism = [(i, exp[i], got[i]) for i in range(len(recs)) if (got[i] == 1) != (exp[i] == -2) or got[i] == 2]
    assert not mism, mism[:10]
    assert 0 < sum(1 for e in exp if e == -2) < len(exp)


def test_second_pass_continues_after_unsupported_set():
    """a set the second pass cannot follow (9-deep nesting) does
    not stop the request walk: a corrupt gzip set after it still fails the
    request (-2, as ReadRequest would); with valid sets after it the result
    stays unsupported (2); the 9-deep value inside a multi-message set does
    not hide a corrupt message after it in the same set."""
    lib = _kcodec()
    deep = C.deep_nesting(9)  # a ProduceReq: take its message set back out
    v = K.gzip_member(C.INNER)
    for _ in range(8):
        v = K.gzip_member(K.wrapper_set(v, K.GZIP, 1))
    deep_set = K.wrapper_set(v, K.GZIP, 1)
    ok = K.gzip_member(C.INNER)
    corrupt_set = K.wrapper_set(ok[:-2], K.GZIP, 1)
    good_set = K.wrapper_set(ok, K.GZIP, 1)
    r_bad = K.produce(1, "c", [("t", [(0, deep_set), (1, corrupt_set)])])
    r_good = K.produce(1, "c", [("t", [(0, deep_set)]), ("u", [(0, good_set)])])
    r_same = K.produce(1, "c", [("t", [(0, deep_set + corrupt_set)])])
    assert _oracle([r_bad, r_good, r_same]) == [-2, -1, -2]  # r_good decodes; topic u is not covered
    assert lib.kc_host_check_produce(r_bad, len(r_bad), SLAB) == 1
    assert lib.kc_host_check_produce(r_good, len(r_good), SLAB) == 2
    assert lib.kc_host_check_produce(r_same, len(r_same), SLAB) == 1
    assert deep  # the 9-deep request itself is covered by test_device_decoder_nesting_and_slab_limits


def test_second_pass_decode_budget_bounds_a_gzip_bomb():
    """a ProduceReq of many small gzip values that each inflate
    to ~6 MB (a gzip bomb) is bounded by the per-request decode budget
    (2 x maxParseBufSize): past it values are unsupported (reported, not
    decoded); a corrupt value met within the budget still fails the request."""
    import time
    lib = _kcodec()
    bomb = K.gzip_member(K.message_set(["a" * 6_000_000], version=1), level=9)
    assert len(bomb) < 64 * 1024
    sets = [K.wrapper_set(bomb, K.GZIP, 1) for _ in range(12)]
    rec = K.produce(1, "c", [("t", [(i, s) for i, s in enumerate(sets)])])
    t = time.perf_counter()
    assert lib.kc_host_check_produce(rec, len(rec), SLAB) == 2
    budget_s = time.perf_counter() - t
    rec_bad = K.produce(1, "c", [("t", [(99, K.wrapper_set(bomb[:-3], K.GZIP, 1))] +
                                  [(i, s) for i, s in enumerate(sets)])])
    assert lib.kc_host_check_produce(rec_bad, len(rec_bad), SLAB) == 1
    # 12 bombs = 72 MB decoded without the budget; with it ~13 MB
    one = K.produce(1, "c", [("t", [(0, sets[0])])])
    t = time.perf_counter()
    assert lib.kc_host_check_produce(one, len(one), SLAB) == 0
    one_s = time.perf_counter() - t
    assert budget_s < 4 * one_s + 0.5, (budget_s, one_s)
