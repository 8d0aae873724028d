"""Synthetic workloads of BASELINE.json's configurations (libl7gen.so).

Request i of a workload depends only on (config, seed, i), so shards of one
workload generated on different ranks concatenate to exactly the single-GPU
batch.  Shapes follow SURVEY.md §8(d)."""
import ctypes
import os

import numpy as np

from . import l7match as L

_HERE = os.path.dirname(os.path.abspath(__file__))
GEN_PATH = os.path.join(_HERE, "libl7gen.so")

CONFIGS = {
    1: dict(name="readme-http-1rule", seed=0xC1, n_rules=1, n_requests=1_000_000, proto=L.PROTO_HTTP),
    2: dict(name="http-1k-rules", seed=0xC2, n_rules=1000, n_requests=64_000_000, proto=L.PROTO_HTTP),
    3: dict(name="kafka-10k-rules", seed=0xC3, n_rules=10000, n_requests=64_000_000, proto=L.PROTO_KAFKA),
    # Config 4 is two generators under one seed: 5k config-2 HTTP rules + 5k
    # config-3 Kafka rules, 128M requests in total (half per protocol), see
    # mixed_parts().  SURVEY.md §8(d) config 4.
    4: dict(name="mixed-http-kafka-10k-rules", seed=0xC4, n_rules=10_000, n_requests=128_000_000, proto=None,
            parts=((2, 5000), (3, 5000))),
    5: dict(name="adversarial-100k-rules", seed=0xC5, n_rules=100_000, n_requests=1_000_000, proto=L.PROTO_HTTP),
}


# HTTP rules with the ECMAScript constructs beyond the regular core that the
# reference accepts (std::regex via Envoy, envoy/cilium_network_policy.h:52-56;
# patterns passed verbatim by pkg/envoy/server.go:276-289): word-delimited API
# versions, "anything but admin", extension filters, repeated path segments.
# bench.py --extended puts them in front of config 2's rules (indices 0..9, so
# they decide first); the back-reference rules send every request whose
# superset automaton matches through the slow pass.
EXTENDED_RULES = [
    L.PortRuleHTTP(Path=".*\\bv1\\b.*", Method="GET"),
    L.PortRuleHTTP(Path="^(?!.*admin).*$", Method="POST"),
    L.PortRuleHTTP(Path="/files/(?!secret)\\w+(\\.\\w+)?"),
    L.PortRuleHTTP(Path=".*\\.(?!exe$)\\w+", Method="PUT"),
    L.PortRuleHTTP(Path="/(?=[a-z]+/)[a-z]+/\\w*\\b"),
    L.PortRuleHTTP(Method="(?!DELETE)[A-Z]+", Path="/ro/.*"),
    L.PortRuleHTTP(Host="(?=.*\\.local$)svc\\d+\\..*"),
    L.PortRuleHTTP(Path="/svc\\d+/v\\d+\\B.*", Headers=["x-tenant: t1"]),
    L.PortRuleHTTP(Path="/(\\w+)/\\1(/.*)?"),                 # repeated segment (back-reference)
    L.PortRuleHTTP(Path="/(a|bb)+-\\1"),                      # back-reference after a loop
]


def _load():
    if not os.path.exists(GEN_PATH):
        raise ImportError(f"{GEN_PATH} missing: make -C cilium_amd/csrc")
    g = ctypes.CDLL(GEN_PATH)
    g.l7g_rules_text.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32]
    g.l7g_rules_text.restype = ctypes.c_char_p
    g.l7g_requests.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                               ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                               ctypes.c_int]
    g.l7g_requests.restype = ctypes.c_uint64
    g.l7g_block_bytes.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                  ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    g.l7g_block_bytes.restype = None
    return g


_gen = _load()


def rules(config: int, seed: int = None, n_rules: int = None):
    c = CONFIGS[config]
    seed = c["seed"] if seed is None else seed
    n_rules = c["n_rules"] if n_rules is None else n_rules
    text = _gen.l7g_rules_text(config, seed, n_rules).decode()
    out = []
    for line in text.splitlines():
        f = line.split("\t")
        if c["proto"] == L.PROTO_HTTP:
            hdrs = [h for h in f[3].split("\x1f") if h] if len(f) > 3 else []
            out.append(L.PortRuleHTTP(Path=f[0], Method=f[1], Host=f[2], Headers=hdrs))
        else:
            out.append(L.PortRuleKafka(Role=f[0], APIKey=f[1], APIVersion=f[2], ClientID=f[3], Topic=f[4]))
    return out


def requests(config: int, start: int, count: int, seed: int = None, n_rules: int = None,
             threads: int = 8, out_arena: np.ndarray = None):
    """Generate requests [start, start+count) -> (arena uint8[], offsets uint64[])."""
    c = CONFIGS[config]
    seed = c["seed"] if seed is None else seed
    n_rules = c["n_rules"] if n_rules is None else n_rules
    size = _gen.l7g_requests(config, seed, n_rules, start, count, None, 0, None, threads)
    if out_arena is None:
        arena = np.empty(size + 64, dtype=np.uint8)
    else:
        arena = out_arena
        assert arena.nbytes >= size
    offs = np.empty(count, dtype=np.uint64)
    used = _gen.l7g_requests(config, seed, n_rules, start, count, arena.ctypes.data, arena.nbytes,
                             offs.ctypes.data, threads)
    assert used == size
    return arena[: size + 64] if out_arena is None else arena, offs


def block_bytes(config: int, start: int, count: int, block: int, seed: int = None, n_rules: int = None,
                threads: int = 8) -> np.ndarray:
    """Record bytes of requests [start, start+count) summed per `block` records
    (sizes only): the input of byte-balanced shard bounds (dist.py)."""
    c = CONFIGS[config]
    seed = c["seed"] if seed is None else seed
    n_rules = c["n_rules"] if n_rules is None else n_rules
    out = np.zeros((count + block - 1) // block, dtype=np.uint64)
    if count:
        _gen.l7g_block_bytes(config, seed, n_rules, start, count, block, out.ctypes.data, threads)
    return out


def mixed_parts(config: int = 4):
    """Config 4 split by protocol tag: [(proto, generator config, seed, n_rules)].

    In Cilium the two protocols never share a call site — HTTP verdicts are
    taken in Envoy's filter (envoy/cilium_l7policy.cc), Kafka verdicts in the
    Go proxy (pkg/proxy/kafka.go) — so a mixed batch is demultiplexed by its
    protocol tag into one arena per protocol, each evaluated against its own
    compiled rule set; request i of part p is request i of generator
    config p under the mixed workload's seed."""
    c = CONFIGS[config]
    return [(CONFIGS[g]["proto"], g, c["seed"], n) for g, n in c["parts"]]
