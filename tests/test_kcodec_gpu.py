"""Compressed Kafka message sets on the GPU (first pass queues gzip / snappy
values, kafka_codec_kernel decodes and re-reads them): bit-exact verdicts and
counters against the oracle for the reference-semantics cases
(tests/kafka_codec_cases.py), random corruptions, a batch mixing compressed
and plain requests at scale, and the explicit nesting limit (-3)."""
import random

import numpy as np
import pytest

import kafka_codec_cases as C
import kafka_wire as K
from cilium_amd import dist as D
from cilium_amd import l7match as L
from cilium_amd import workloads as W
from oracle import KafkaOracle

pytestmark = pytest.mark.gpu


def _check(rules, recs, exp_list=None):
    arena, offs = L.pack_records(recs)
    rs = L.RuleSet.compile_kafka(rules)
    h = np.zeros(rs.n_counters, dtype=np.uint64)
    got = rs.eval(arena, offs, h)
    exp = KafkaOracle(rules).eval(arena, offs, threads=8)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]
    assert np.array_equal(h, D.counters_from_verdicts(got, len(rules)))
    if exp_list is not None:
        assert got.tolist() == exp_list
    return got


def test_compressed_cases_gpu(gpu):
    cases = C.request_cases()
    _check([L.PortRuleKafka(Topic="t")], [c[1] for c in cases], [c[2] for c in cases])
    deny = C.deny_cases()
    _check([L.PortRuleKafka(Topic="x")], [c[1] for c in deny], [c[2] for c in deny])


def test_compressed_random_corruptions_gpu(gpu):
    rnd = random.Random(11)
    base = [(K.GZIP, K.gzip_member(C.INNER)), (K.SNAPPY, K.snappy_block(C.INNER)),
            (K.SNAPPY, K.snappy_java(C.INNER, chunk=33)), (K.GZIP, K.gzip_member(C.INNER, level=0))]
    recs = []
    for i in range(4000):
        codec, v = rnd.choice(base)
        v = bytearray(v)
        if i % 4:
            v[rnd.randrange(len(v))] ^= 1 << rnd.randrange(8)
        recs.append(K.produce(1 + i % 3, "c", [("t", [(0, K.wrapper_set(bytes(v), codec, 1 + i % 3))])]))
    v = _check([L.PortRuleKafka(Topic="t")], recs)
    assert (v == 0).any() and (v == -2).any()


def test_mixed_batch_with_compressed_requests_gpu(gpu):
    """Config-3 traffic with every 7th request replaced by a compressed
    produce request (valid or corrupt): verdicts and counters bit-exact."""
    rules = W.rules(3, n_rules=2000)
    arena, offs = W.requests(3, 0, 30_000, n_rules=2000)
    buf = arena.tobytes()
    recs = []
    for i, o in enumerate(offs.tolist()):
        n = int.from_bytes(buf[o:o + 4], "big") + 4
        recs.append(buf[o:o + n])
    ok = K.gzip_member(C.INNER)
    for i in range(0, len(recs), 7):
        val = ok if i % 2 else ok[:-1]
        recs[i] = K.produce(2, f"client-{i % 100}", [(f"topic-{i % 2000}", [(0, K.wrapper_set(val, K.GZIP, 2))])])
    v = _check(rules, recs)
    assert (v == -2).sum() >= len(recs) // 14 - 1


def test_nesting_limit_reports_unsupported(gpu):
    """The second pass follows 8 nested compressed sets; a 9th is reported as
    L7M_VERDICT_UNSUPPORTED (the oracle, with no limit, allows it)."""
    recs = [C.deep_nesting(8), C.deep_nesting(9)]
    arena, offs = L.pack_records(recs)
    rs = L.RuleSet.compile_kafka([L.PortRuleKafka(Topic="t")])
    assert rs.eval(arena, offs).tolist() == [0, L.VERDICT_UNSUPPORTED]
    assert KafkaOracle([L.PortRuleKafka(Topic="t")]).eval(arena, offs).tolist() == [0, 0]


def test_random_multi_partition_produce_requests_gpu(gpu):
    """Produce requests of several topics / partitions mixing plain and
    compressed messages, corrupt values and sets that end early (bad CRC,
    attribute 3, truncated message: the rest of the set is read as the next
    partition's fields): verdicts and counters bit-exact with the oracle."""
    recs = C.random_produce_requests(random.Random(23), 3000, framing_stops=True)
    v = _check([L.PortRuleKafka(Topic="t")], recs)
    assert (v == 0).any() and (v == -1).any() and (v == -2).any()


def test_batcher_resident_kafka_codec_fallback(gpu):
    """Through the batcher, Kafka batches go to the resident workgroup; a
    batch holding a compressed message set is handed back (the resident
    workgroup has no codec queue) and evaluated by the normal launches with
    the second pass: verdicts equal the oracle's for a mix of plain and
    compressed / corrupt produce requests called from 8 threads."""
    import threading
    recs = C.random_produce_requests(random.Random(29), 600, framing_stops=True)
    rules = [L.PortRuleKafka(Topic="t")]
    arena, offs = L.pack_records(recs)
    exp = KafkaOracle(rules).eval(arena, offs)
    b = L.Batcher(L.RuleSet.compile_kafka(rules), max_delay_us=100, in_flight=3)
    got = np.full(len(recs), -100, dtype=np.int64)

    def worker(t):
        for i in range(t, len(recs), 8):
            got[i] = b.eval(recs[i])

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    b.close()
    assert np.array_equal(got, exp)
    assert (exp == -2).any() and (exp == 0).any()
