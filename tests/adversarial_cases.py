"""Constructed long-field requests for BASELINE config 5's rule families
(cilium_amd/csrc/l7gen.cc adv_path_rule): paths and header values up to the
record format's 64 KiB field limit, each with the verdict its construction
implies.  The expected verdicts are derived from the patterns' languages by
hand (not by any engine), so they pin the NFA oracle (oracle/nfa.h) and the
GPU on inputs std::regex cannot evaluate.

Families (rule i):
  i % 5 == 0  /a{i}/(a|aa)*b
  i % 5 == 1  /x{i}/.*(x|y).*(z|w).*q
  i % 5 == 2  /l{i}/(w0|...|w99)
  i % 5 == 3  /c{i}/[a-z]*[a-z]*[a-z]*[a-z]*z
  i % 5 == 4  /f{i}/(.{0,8}){1,8}foo      ((.{0,8}){1,8} = any 0..64 non-CR/LF bytes)
Rules with i % 97 == 0 also need the literal header x-blob (avoided here
except in the dedicated blob cases)."""
import random
import struct

import numpy as np

from cilium_amd import l7match as L

MAX_FIELD = 65535


def _words(rule_path):
    inner = rule_path[rule_path.index("(") + 1:rule_path.rindex(")")]
    return inner.split("|")


def long_field_cases(rules, n, seed=5):
    """[(HTTPRequest, expected verdict)] for n constructed requests."""
    rng = random.Random(seed)
    n_rules = len(rules)
    out = []
    while len(out) < n:
        i = rng.randrange(n_rules)
        if i % 97 == 0:
            continue
        fam = i % 5
        pre = rules[i].Path.split("/")[1]
        head = "/" + pre + "/"
        long_len = rng.choice([100, 1000, 8000, 9000, 30000, MAX_FIELD - len(head) - 8])
        good = rng.random() < 0.5
        if fam == 0:
            tail = "a" * long_len + ("b" if good else "c")
        elif fam == 1:
            # good: an x, later a z, a q at the end; bad: no z/w after the only x/y
            fill = "".join(rng.choice("xyzwq.") for _ in range(long_len))
            tail = ("x" + fill[:long_len - 60] + "z" + fill[:50] + "q") if good else ("w" * long_len + "y.q")
        elif fam == 2:
            w = rng.choice(_words(rules[i].Path))
            tail = w if good else (w * (long_len // max(1, len(w)) + 2))[:long_len]
        elif fam == 3:
            fill = "".join(rng.choice("abcdefghijklmnopqrstuvwxyz") for _ in range(long_len))
            tail = fill + ("z" if good else "y")
        else:
            k = min(rng.choice([0, 1, 60, 61, 62, 64, 65, 70, 500, long_len]), MAX_FIELD - len(head) - 3)
            fill = "".join(rng.choice("abfo.") for _ in range(k))
            tail = fill + ("foo" if good else "fob")
            good = good and k <= 64
        path = head + tail
        assert len(path) <= MAX_FIELD
        hdrs = [("x-filler", "v" * rng.choice([0, 10, 2000]))]
        if rng.random() < 0.3:
            hdrs.append(("x-blob", "".join(rng.choice("abc123") for _ in range(rng.choice([1024, 20000, 65535])))))
        req = L.HTTPRequest(method="GET", path=path, authority="adv.example", headers=hdrs)
        out.append((req, i if good else L.VERDICT_DENY))
    return out


def blob_cases(rules, n, seed=7):
    """x-blob literal-header rules (i % 97 == 0): exact value allows (when the
    path matches too), a one-byte change or a longer value denies."""
    rng = random.Random(seed)
    out = []
    blob_rules = [i for i in range(len(rules)) if i % 97 == 0]
    for _ in range(n):
        i = rng.choice(blob_rules)
        r = rules[i]
        val = next(h for h in r.Headers if h.startswith("x-blob"))[len("x-blob: "):]
        pre = r.Path.split("/")[1]
        fam = i % 5  # the family's shortest matching tail
        tail = {0: "b", 1: "xzq", 2: _words(r.Path)[0] if fam == 2 else "", 3: "z", 4: "foo"}[fam]
        path = "/" + pre + "/" + tail
        mode = rng.randrange(3)
        if mode == 0:
            v, exp = val, i
        elif mode == 1:
            k = rng.randrange(len(val))
            v, exp = val[:k] + ("#" if val[k] != "#" else "$") + val[k + 1:], L.VERDICT_DENY
        else:
            v, exp = val + "x" * rng.choice([1, 5000, 60000]), L.VERDICT_DENY
        req = L.HTTPRequest(method="GET", path=path, authority="adv.example", headers=[("x-blob", v[:MAX_FIELD])])
        out.append((req, exp))
    return out


def cheap_for_oracle(arena, offs, max_f_tail=24):
    """Mask of records whose path std::regex evaluates quickly: `/f{i}/` tails
    <= max_f_tail bytes ((.{0,8}){1,8}foo backtracks exponentially beyond)."""
    buf = arena.tobytes()
    keep = np.ones(len(offs), dtype=bool)
    for i, o in enumerate(offs.tolist()):
        w2, w3 = struct.unpack_from("<II", buf, o + 8)
        nh, ml, pl = w2 >> 24, w3 & 0xFFFF, w3 >> 16
        p = o + 20 + 4 * nh + ml
        path = buf[p:p + pl]
        if path.startswith(b"/f"):
            k = path.find(b"/", 1)
            keep[i] = k < 0 or pl - k - 1 <= max_f_tail
    return keep


def subset(arena, offs, keep):
    """Re-pack the records selected by a mask."""
    recs = []
    buf = arena.tobytes()
    for o in offs[keep].tolist():
        ln = struct.unpack_from("<I", buf, o)[0]
        recs.append(buf[o:o + ((ln + 3) & ~3)])
    return L.pack_records(recs)
