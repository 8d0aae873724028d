"""Verdict side effects on the host (no GPU): the 403 body
(envoy/cilium_l7policy.cc:89-95), the Kafka deny response
CreateResponse(ErrTopicAuthorizationFailed) serialised as optiopay's
Resp.Bytes(version) for every request kind / version the decoder types
(checked against the test-side restatement kafka_wire.deny_response), and the
per-endpoint proxy statistics."""
import struct

import numpy as np
import pytest

import kafka_wire as K
from cilium_amd import l7match as L


def test_http_deny_body():
    assert L.http_deny_body("") == b"Access denied\r\n"
    assert L.http_deny_body("Nope") == b"Nope\r\n"
    assert L.http_deny_body("Nope\r\n") == b"Nope\r\n"
    assert L.http_deny_body("\n") == b"\n\r\n"        # len < 2: CRLF appended
    assert L.http_deny_body("a\r") == b"a\r\r\n"


TOPICS = [("t1", [0, 3]), ("topic-two", [7])]


def _cases():
    ms = K.message_set(["v"], version=1)
    for v in range(4):
        yield (f"produce_v{v}", K.produce(v, "c", [(n, [(p, ms) for p in ps]) for n, ps in TOPICS]),
               K.deny_response(K.PRODUCE, v, 1, TOPICS))
    for v in range(6):
        yield f"fetch_v{v}", K.fetch(v, "c", TOPICS), K.deny_response(K.FETCH, v, 1, TOPICS)
    for v in range(3):
        yield f"offsets_v{v}", K.offsets(v, "c", TOPICS), K.deny_response(K.OFFSETS, v, 1, TOPICS)
    for v in range(5):
        names = [n for n, _ in TOPICS]
        yield f"metadata_v{v}", K.metadata(v, "c", names), K.deny_response(K.METADATA, v, 1, names)
        yield f"metadata_all_v{v}", K.metadata(v, "c", []), K.deny_response(K.METADATA, v, 1, [])
    for v in range(3):
        yield (f"offset_commit_v{v}", K.offset_commit(v, "c", "g", TOPICS),
               K.deny_response(K.OFFSET_COMMIT, v, 1, TOPICS))
    for v in range(3):
        yield (f"offset_fetch_v{v}", K.offset_fetch(v, "c", "g", TOPICS),
               K.deny_response(K.OFFSET_FETCH, v, 1, TOPICS))
    for v in range(2):
        yield (f"consumer_metadata_v{v}", K.consumer_metadata(v, "c", "g"),
               K.deny_response(K.CONSUMER_METADATA, v, 1, []))


@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_kafka_deny_response(case):
    _, req, exp = case
    assert L.kafka_deny_response(req) == exp


def test_kafka_deny_response_reference_proxy_case():
    """pkg/proxy/kafka_test.go:252-258: producing to a disallowed topic gets a
    ProduceResp whose partition carries ErrTopicAuthorizationFailed (29) and
    the request's correlation id."""
    req = K.produce(0, "client", [("disallowedTopic", [(0, K.message_set(["Message 1"]))])])
    req = req[:8] + struct.pack(">i", 4242) + req[12:]
    resp = L.kafka_deny_response(req)
    size, corr, nt = struct.unpack_from(">iii", resp, 0)
    assert size == len(resp) - 4 and corr == 4242 and nt == 1
    off = 12 + 2 + len("disallowedTopic")
    np_, pid, err = struct.unpack_from(">iih", resp, off)
    assert (np_, pid, err) == (1, 0, 29)


def test_kafka_deny_response_follows_message_set_consumption():
    """readMessageSet can stop inside a set (attributes 3): the next partition
    of the request is read from there, as the reference does."""
    stop = K.message_set(["z"], version=1, compression=3)
    tail = struct.pack(">ii", 9, 0)  # read as the next partition's id and set size
    req = K.produce(1, "c", [("t", [(5, stop + tail)])])
    # the set claims len(stop + tail) bytes, but reading stops after `stop`;
    # the request's partition array then ends (np = 1): nothing more is read
    assert L.kafka_deny_response(req) == K.deny_response(K.PRODUCE, 1, 1, [("t", [5])])


def test_kafka_deny_response_errors():
    with pytest.raises(L.L7Error) as e:
        L.kafka_deny_response(K.generic(18, 0))      # ApiVersions: request == nil
    assert e.value.code == L.L7M_EUNSUPPORTED
    with pytest.raises(L.L7Error) as e:
        L.kafka_deny_response(K.fetch(0, "c", TOPICS)[:30])
    assert e.value.code == L.L7M_EINVAL


def test_proxy_stats():
    v = np.array([0, 5, -1, -1, -2, -3, 7], dtype=np.int32)
    assert L.proxy_stats(v) == {"received": 7, "forwarded": 3, "denied": 2, "error": 2}


# ---------------------------------------------------------------- access log --
def _http_log_entry_class():
    """cilium.HttpLogEntry built from envoy/cilium/accesslog.proto's field
    numbers and types (transcribed schema; the library's bytes must parse and
    re-serialize identically with the protobuf runtime)."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fp = descriptor_pb2.FileDescriptorProto(name="l7m_test_accesslog.proto", package="cilium", syntax="proto3")
    kv = fp.message_type.add(name="KeyValue")
    kv.field.add(name="key", number=1, type=F.TYPE_STRING, label=F.LABEL_OPTIONAL)
    kv.field.add(name="value", number=2, type=F.TYPE_STRING, label=F.LABEL_OPTIONAL)
    e = fp.message_type.add(name="HttpLogEntry")
    for name, num, typ in [("timestamp", 1, F.TYPE_UINT64), ("http_protocol", 2, F.TYPE_UINT32),
                           ("entry_type", 3, F.TYPE_UINT32), ("policy_name", 4, F.TYPE_STRING),
                           ("cilium_rule_ref", 5, F.TYPE_STRING), ("source_security_id", 6, F.TYPE_UINT32),
                           ("source_address", 7, F.TYPE_STRING), ("destination_address", 8, F.TYPE_STRING),
                           ("scheme", 9, F.TYPE_STRING), ("host", 10, F.TYPE_STRING), ("path", 11, F.TYPE_STRING),
                           ("method", 12, F.TYPE_STRING), ("status", 13, F.TYPE_UINT32)]:
        e.field.add(name=name, number=num, type=typ, label=F.LABEL_OPTIONAL)
    e.field.add(name="headers", number=14, type=F.TYPE_MESSAGE, type_name=".cilium.KeyValue",
                label=F.LABEL_REPEATED)
    e.field.add(name="is_ingress", number=15, type=F.TYPE_BOOL, label=F.LABEL_OPTIONAL)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fp)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("cilium.HttpLogEntry"))


def test_http_access_log_entries():
    """AccessLog::Entry::InitFromRequest / UpdateFromResponse / Log
    (envoy/accesslog.cc:59-170) as AccessFilter drives them
    (cilium_l7policy.cc:166-191): Request entries for allowed requests,
    Denied + 403 for denied ones; x-forwarded-proto -> scheme; other headers
    in order; identity by direction."""
    Entry = _http_log_entry_class()
    reqs = [L.HTTPRequest("GET", "/public/a", "svc.local", [("x-forwarded-proto", "https"), ("x-token", "12"),
                                                            ("x-a", "1"), ("x-a", "2")], remote_id=7, ingress=True),
            L.HTTPRequest("POST", "/private", None, [("user-agent", "curl")], remote_id=9, dport=8080, ingress=False),
            L.HTTPRequest(None, None, None, [], remote_id=1)]
    arena, offs = L.pack_http(reqs)
    verdicts = np.array([3, L.VERDICT_DENY, L.VERDICT_ALLOW_NO_L7], dtype=np.int32)
    msgs = L.http_access_log(arena, offs, verdicts, policy_name="ep-1", timestamp_ns=1_500_000_000_123,
                             local_identity=4242, source_address="10.0.0.1:4000")
    assert len(msgs) == 3
    e = [Entry.FromString(m) for m in msgs]
    for m, x in zip(msgs, e):
        assert x.SerializeToString() == m  # canonical encoding (field order, proto3 defaults)
    assert e[0].entry_type == 0 and e[0].status == 0 and e[0].is_ingress
    assert (e[0].method, e[0].path, e[0].host, e[0].scheme) == ("GET", "/public/a", "svc.local", "https")
    assert [(h.key, h.value) for h in e[0].headers] == [("x-token", "12"), ("x-a", "1"), ("x-a", "2")]
    assert e[0].source_security_id == 7 and e[0].policy_name == "ep-1" and e[0].http_protocol == 1
    assert e[0].timestamp == 1_500_000_000_123 and e[0].source_address == "10.0.0.1:4000"
    assert e[0].cilium_rule_ref == ""  # this reference's filter does not set it
    assert e[1].entry_type == 2 and e[1].status == 403 and not e[1].is_ingress
    assert e[1].source_security_id == 4242  # egress: the local endpoint is the source
    assert e[1].host == "" and [(h.key, h.value) for h in e[1].headers] == [("user-agent", "curl")]
    assert e[2].method == "" and e[2].path == "" and e[2].entry_type == 0


def test_kafka_access_log_records():
    """kafkaLogRecord.log (pkg/proxy/kafka.go:168-230): one record per topic,
    Forwarded/0 or Denied/29, apiKeyToString names; no record for requests
    without topics or that ReadRequest rejects."""
    recs = [K.produce(2, "cli", [("t1", [(0, b"")]), ("t2", [(1, b"")])]),
            K.metadata(1, "cli", ["m1"]),
            K.metadata(0, "cli", []),
            K.consumer_metadata(0, "cli", "grp"),
            K.generic(18, 0),
            b"\x00\x00\x00\x02\x00\x00"]
    arena, offs = L.pack_records(recs)
    verdicts = np.array([0, L.VERDICT_DENY, 1, 2, L.VERDICT_DENY, L.VERDICT_PARSE_ERROR], dtype=np.int32)
    out = L.kafka_access_log(arena, offs, verdicts)
    assert [(r["request"], r["verdict"], r["error_code"], r["api_key"], r["api_version"], r["topic"]) for r in out] == [
        (0, "Forwarded", 0, "produce", 2, "t1"), (0, "Forwarded", 0, "produce", 2, "t2"),
        (1, "Denied", 29, "metadata", 1, "m1")]
    assert all(r["correlation_id"] == 1 for r in out)
    assert L.kafka_api_key_name(18) == "apiversions" and L.kafka_api_key_name(-5) == "-5"


def test_proxy_stats_keyed_like_the_endpoint():
    """UpdateProxyStatistics(l7Protocol, port, ingress, request, verdict)
    (pkg/endpoint/endpoint.go:2099-2122): HTTP keyed by each record's dport and
    direction, Kafka by the redirect's; Kafka port 0 and parse errors are not
    counted."""
    t = L.ProxyStatsTable()
    reqs = [L.HTTPRequest("GET", "/", dport=80, ingress=True), L.HTTPRequest("GET", "/", dport=80, ingress=True),
            L.HTTPRequest("GET", "/", dport=8080, ingress=False)]
    arena, offs = L.pack_http(reqs)
    t.update(L.PROTO_HTTP, arena, offs, np.array([0, L.VERDICT_DENY, L.VERDICT_ALLOW_NO_PORT_POLICY], np.int32))
    karena, koffs = L.pack_records([K.metadata(0, "c", ["x"])] * 4)
    kv = np.array([0, L.VERDICT_DENY, L.VERDICT_PARSE_ERROR, L.VERDICT_UNSUPPORTED], np.int32)
    t.update(L.PROTO_KAFKA, karena, koffs, kv, port=9092, ingress=True)
    t.update(L.PROTO_KAFKA, karena, koffs, kv, port=0, ingress=True)
    e = t.entries()
    assert e == {("http", 80, True, True): {"received": 2, "forwarded": 1, "denied": 1, "error": 0},
                 ("http", 8080, False, True): {"received": 1, "forwarded": 1, "denied": 0, "error": 0},
                 ("kafka", 9092, True, True): {"received": 3, "forwarded": 1, "denied": 1, "error": 1}}


def test_proxy_stats_denied_untyped_kafka_kind_is_error():
    """A denied request of a kind ReadRequest leaves untyped (heartbeat = 12,
    request == nil) cannot get its deny response: CreateResponse fails
    (pkg/kafka/request.go:174-175) and handleRequest logs VerdictError
    (pkg/proxy/kafka.go:246-252), so the endpoint counts an error; an allowed
    one is forwarded, a denied typed one is denied."""
    t = L.ProxyStatsTable()
    recs = [K.generic(12, 0, "c"), K.generic(12, 0, "c"), K.metadata(0, "c", ["x"])]
    arena, offs = L.pack_records(recs)
    t.update(L.PROTO_KAFKA, arena, offs, np.array([L.VERDICT_DENY, 0, L.VERDICT_DENY], np.int32), port=9092,
             ingress=False)
    assert t.entries() == {("kafka", 9092, False, True): {"received": 3, "forwarded": 1, "denied": 1, "error": 1}}
