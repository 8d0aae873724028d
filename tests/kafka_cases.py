"""Kafka known-answer batches built from tests/golden/kafka_known_answers.json
(transcribed from the reference's own tests; see tests/golden/make_golden.py).
Each case is (name, rules, records, expected_verdicts)."""
import json
import os

import kafka_wire as K
from cilium_amd import l7match as L

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kafka_known_answers.json")
LOREM = ("Lorem ipsum dolor sit amet, consectetur adipiscing elit. Donec a diam lectus. Sed sit amet ipsum "
         "mauris. Maecenas congue ligula ac quam viverra nec consectetur ante hendrerit.")


def golden():
    with open(GOLD) as f:
        return json.load(f)


def rule(d):
    return L.PortRuleKafka(Role=d.get("Role", ""), APIKey=d.get("APIKey", ""), APIVersion=d.get("APIVersion", ""),
                           ClientID=d.get("ClientID", ""), Topic=d.get("Topic", ""))


def _req_record(q, msgs=("first", "second")):
    kind, ver = q["kind"], q["version"]
    if kind == K.PRODUCE:
        ms = K.message_set(list(msgs), version=ver)
        return K.produce(ver, q["client"], [(t, [(0, ms)]) for t in q["topics"]])
    if kind == K.METADATA:
        return K.metadata(ver, q["client"], q["topics"])
    return K.generic(kind, ver, q.get("client", ""))


def cases():
    g = golden()
    out = []
    pt = g["policy_test"]
    rec = _req_record(pt["request"], msgs=[LOREM] * 3)
    for i, c in enumerate(pt["cases"]):
        exp = c["verdict"] if c["allow"] else L.VERDICT_DENY
        out.append((f"policy_test[{i}]", [rule(r) for r in c["rules"]], [rec], [exp]))
    for i, c in enumerate(g["unknown_kind"]["cases"]):
        exp = c["verdict"] if c["allow"] else L.VERDICT_DENY
        out.append((f"unknown_kind[{i}]", [rule(r) for r in c["rules"]], [K.generic(c["kind"], 0)], [exp]))
    px = g["proxy"]
    recs = [_req_record(c["req"]) for c in px["cases"]]
    exps = [c["verdict"] if c["allow"] else L.VERDICT_DENY for c in px["cases"]]
    out.append(("proxy", [rule(r) for r in px["rules"]], recs, exps))
    return out
