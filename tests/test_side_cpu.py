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
