"""CPU tests of the Kafka path: the oracle pinned to the reference's own known
answers, Sanitize parity between the product compiler (l7m_compile_kafka) and
the oracle, and the wire encoder used by the GPU tests.  No GPU calls."""
import numpy as np
import pytest

import kafka_wire as K
from cilium_amd import l7match as L
from cilium_amd import workloads as W
from kafka_cases import cases, golden, rule
from oracle import KafkaOracle, OracleError


@pytest.mark.parametrize("name,rules,records,expected", cases(), ids=[c[0] for c in cases()])
def test_oracle_reference_known_answers(name, rules, records, expected):
    arena, offs = L.pack_records(records)
    assert KafkaOracle(rules).eval(arena, offs).tolist() == expected


def test_sanitize_known_answers_compiler_and_oracle_agree():
    for c in golden()["sanitize"]["cases"]:
        r = rule(c["rule"])
        if c["ok"]:
            L.RuleSet.compile_kafka([r])
            KafkaOracle([r])
        else:
            with pytest.raises(L.L7Error) as e:
                L.RuleSet.compile_kafka([r])
            assert e.value.code == L.L7M_EINVAL_RULE
            with pytest.raises(OracleError):
                KafkaOracle([r])


def test_sanitize_edge_cases():
    ok = [L.PortRuleKafka(APIKey="ApiVersions"), L.PortRuleKafka(APIKey="İnitproducerid"),
          L.PortRuleKafka(Role="PRODUCE"), L.PortRuleKafka(APIVersion="-32768"),
          L.PortRuleKafka(APIVersion="007"), L.PortRuleKafka(Topic="a\\b")]
    bad = [L.PortRuleKafka(APIVersion="1.0"), L.PortRuleKafka(APIVersion=""),  # "" = unset -> ok below
           L.PortRuleKafka(APIVersion="+"), L.PortRuleKafka(APIVersion="32768"),
           L.PortRuleKafka(Topic="té"), L.PortRuleKafka(Topic="a b"), L.PortRuleKafka(APIKey="produce "),
           L.PortRuleKafka(Role="admin")]
    for r in ok:
        L.RuleSet.compile_kafka([r])
        KafkaOracle([r])
    for r in bad:
        if r.APIVersion == "" and r.Topic == "" and r.APIKey == "" and r.Role == "":
            L.RuleSet.compile_kafka([r])
            continue
        with pytest.raises(L.L7Error):
            L.RuleSet.compile_kafka([r])
        with pytest.raises(OracleError):
            KafkaOracle([r])


def test_example_policies_compile():
    ex = golden()["examples"]
    for key in ("rules", "role_rules"):
        rs = L.RuleSet.compile_kafka([rule(r) for r in ex[key]])
        assert rs.n_rules == len(ex[key]) and rs.n_counters == rs.n_rules + 2


def test_oracle_parses_encoder_output():
    rng = np.random.default_rng(3)
    recs = K.random_requests(rng, 3000, ["t%d" % i for i in range(20)], ["c%d" % i for i in range(5)])
    arena, offs = L.pack_records(recs)
    v = KafkaOracle([L.PortRuleKafka()]).eval(arena, offs)
    # the wildcard rule allows every well-formed request
    assert (v == 0).all(), np.unique(v)


def test_oracle_message_set_semantics():
    ms_ok = K.message_set(["a", "bb"], version=0)
    ms_badcrc = K.message_set(["a", "bb"], version=0, bad_crc_at=0)
    ms_gzip = K.message_set(["zz"], version=1, compression=1)
    ms_attr3 = K.message_set(["zz"], version=1, compression=3)
    recs = [K.produce(0, "c", [("t", [(0, ms_ok)])]),
            K.produce(0, "c", [("t", [(0, ms_badcrc)])]),       # CRC mismatch: rest of set left unread
            K.produce(1, "c", [("t", [(0, ms_gzip)])]),         # "zz" is no gzip stream: NewReader fails
            K.produce(1, "c", [("t", [(0, ms_attr3)])]),        # attribute 3: nil, nil
            K.produce(0, "c", [("t", [(0, ms_ok[:-3])])])]      # truncated last message: ignored
    arena, offs = L.pack_records(recs)
    v = KafkaOracle([L.PortRuleKafka(Topic="t")]).eval(arena, offs)
    assert v.tolist() == [0, 0, L.VERDICT_PARSE_ERROR, 0, 0]


def test_config3_generator_and_oracle_sample():
    rules = W.rules(3, n_rules=2000)
    arena, offs = W.requests(3, 0, 5000, n_rules=2000)
    v = KafkaOracle(rules).eval(arena, offs)
    assert (v >= 0).any() and (v == -1).any() and not (v <= -2).any()


def test_l7datamap_oracle_allows_exactly_what_getrelevantrules_allows():
    """The map oracle (rules filtered by the source's selector mask, in
    compiled order) allows or denies exactly as MatchesRule over the list
    GetRelevantRules builds for that source (selecting entries, then the
    wildcard entries appended)."""
    import selector_cases as S
    entries, ids = S.random_map(3, n_rules=600, n_ids=12)
    arena, offs = W.requests(3, 7_000_000, 3000, n_rules=600)
    idv = S.request_identities(5, len(offs), ids)
    got = KafkaOracle.from_map(entries, ids).eval(arena, offs, threads=8, identities=idv)
    for ident in np.unique(idv).tolist():
        sel = np.nonzero(idv == ident)[0]
        sub_a, sub_o = L.pack_records([bytes(arena[offs[i]:(offs[i + 1] if i + 1 < len(offs) else arena.nbytes)])
                                       for i in sel])
        ref = KafkaOracle(S.relevant_rules(entries, ids, ident)).eval(sub_a, sub_o)
        assert np.array_equal(got[sel] >= 0, ref >= 0), ident
        assert np.array_equal(got[sel] <= -2, ref <= -2), ident
    assert (got >= 0).any() and (got == -1).any()


def test_l7datamap_compile_errors():
    r = [L.PortRuleKafka(Topic="t")]
    with pytest.raises(L.L7Error) as e:
        L.RuleSet.compile_kafka_map([(r, False)] * 65)
    assert e.value.code == L.L7M_ETOOBIG
    for ids in ({0: [0]}, {5: [3]}):
        with pytest.raises(L.L7Error) as e:
            L.RuleSet.compile_kafka_map([(r, False), (r, True)], ids)
        assert e.value.code == L.L7M_EINVAL
    L.RuleSet.compile_kafka_map([(r, False), (r, True)], {5: [0]})
    L.RuleSet.compile_kafka_map([], {})
