"""HTTP records built from raw byte strings (include/l7match.h record
layout), so fields may hold NUL and high bytes — l7m_pack_http takes C
strings.  Shared by the CPU (interpreter) and GPU parity tests."""
import struct

import numpy as np

from cilium_amd import l7match as L


def pack_raw(reqs):
    """(method, path, host, [(name, value)]) byte tuples -> (arena, offsets)."""
    recs = []
    for method, path, host, hdrs in reqs:
        flags = 1 | 2 | 4  # method, path, authority present
        body = b"".join(struct.pack("<I", len(n) | len(v) << 16) for n, v in hdrs)
        body += method + path + host + b"".join(n + v for n, v in hdrs)
        size = 20 + len(body)
        rec = struct.pack("<5I", size, 0, 80 | flags << 16 | len(hdrs) << 24, len(method) | len(path) << 16,
                          len(host)) + body
        recs.append(rec + b"\0" * (-len(rec) % 4))
    return L.pack_records(recs)


def nul_high_byte_case(n, seed=41):
    """Rules over NUL / high bytes and n random requests mixing them."""
    rng = np.random.default_rng(seed)
    rules = [L.PortRuleHTTP(Path="/a.*b"), L.PortRuleHTTP(Path="/x\\x00y.*"),
             L.PortRuleHTTP(Path="[\\x00-\\x7f]+", Method="GET"), L.PortRuleHTTP(Host=".*\\.(com|net)"),
             L.PortRuleHTTP(Path="/[\\x80-\\xff]{2,}/.*", Headers=["x-k: v"]),
             L.PortRuleHTTP(Path="\\x00+", Method="POST")]
    pieces = [b"/a", b"b", b"/x\x00y", b"\x00", b"\xff", b"\x80\x81", b"/", b".com", b".net", b"z", b"\x7f"]
    reqs = []
    for _ in range(n):
        path = b"".join(rng.choice(pieces) for _ in range(rng.integers(0, 8)))
        if rng.random() < 0.2:
            path = bytes(rng.integers(0, 256, size=int(rng.integers(0, 24)), dtype=np.uint8))
        host = b"".join(rng.choice(pieces) for _ in range(rng.integers(0, 4)))
        hdrs = [(b"x-k", rng.choice([b"v\x00", b"v", b"\x00"]))] if rng.random() < 0.4 else []
        reqs.append((rng.choice([b"GET", b"POST", b"G\x00T"]), path, host, hdrs))
    arena, offs = pack_raw(reqs)
    return rules, arena, offs
