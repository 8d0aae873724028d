"""Verdict side effects fed from GPU verdicts: the
HttpLogEntry records (envoy/accesslog.cc:59-170), the Kafka proxy's
per-topic log records (pkg/proxy/kafka.go:168-230), the keyed per-endpoint
proxy statistics (pkg/endpoint/endpoint.go:2099-2122) and the Kafka
ErrTopicAuthorizationFailed responses (pkg/kafka/response.go:81-303,
request.go:158-182) of a config-2 and a config-3 batch decided by the
kernels, against the same functions driven by the oracle's verdicts."""
import struct

import numpy as np
import pytest

from cilium_amd import l7match as L
from cilium_amd import workloads as W
from oracle import HttpOracle, KafkaOracle

pytestmark = pytest.mark.gpu


def test_http_side_effects_from_gpu_verdicts(gpu):
    rules = W.rules(2)
    arena, offs = W.requests(2, 7_000_000, 20_000)
    got = L.RuleSet.compile_http(rules).eval(arena, offs)
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    assert np.array_equal(got, exp)
    kw = dict(policy_name="ep-7", timestamp_ns=1_700_000_000_000, local_identity=99, source_address="10.1.2.3:1")
    logs = L.http_access_log(arena, offs, got, **kw)
    assert logs == L.http_access_log(arena, offs, exp, **kw)
    assert len(logs) == len(got)
    t_gpu, t_orc = L.ProxyStatsTable(), L.ProxyStatsTable()
    t_gpu.update(L.PROTO_HTTP, arena, offs, got)
    t_orc.update(L.PROTO_HTTP, arena, offs, exp)
    e = t_gpu.entries()
    assert e == t_orc.entries()
    tot = {k: sum(v[k] for v in e.values()) for k in ("received", "forwarded", "denied", "error")}
    assert tot == {"received": len(got), "forwarded": int((got >= 0).sum()), "denied": int((got == -1).sum()),
                   "error": int((got < -1).sum())}
    assert L.proxy_stats(got) == L.proxy_stats(exp)


def test_kafka_side_effects_from_gpu_verdicts(gpu):
    rules = W.rules(3, n_rules=2000)
    arena, offs = W.requests(3, 7_000_000, 20_000, n_rules=2000)
    got = L.RuleSet.compile_kafka(rules).eval(arena, offs)
    exp = KafkaOracle(rules).eval(arena, offs, threads=8)
    assert np.array_equal(got, exp)
    recs = L.kafka_access_log(arena, offs, got)
    assert recs == L.kafka_access_log(arena, offs, exp)
    assert {r["verdict"] for r in recs} == {"Forwarded", "Denied"}
    t_gpu, t_orc = L.ProxyStatsTable(), L.ProxyStatsTable()
    t_gpu.update(L.PROTO_KAFKA, arena, offs, got, port=9092, ingress=True)
    t_orc.update(L.PROTO_KAFKA, arena, offs, exp, port=9092, ingress=True)
    assert t_gpu.entries() == t_orc.entries()
    buf = arena.tobytes()
    denied = np.nonzero(got == L.VERDICT_DENY)[0]
    assert len(denied) > 100
    for i in denied[:500].tolist():
        o = int(offs[i])
        n = 4 + struct.unpack_from(">I", buf, o)[0]
        resp = L.kafka_deny_response(buf[o:o + n])
        # the response carries the request's correlation id and its own size
        assert struct.unpack_from(">I", resp, 0)[0] == len(resp) - 4
        assert resp[4:8] == buf[o + 8:o + 12]
