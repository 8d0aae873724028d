"""Files exchanged with tests/cpp/bin/abi_harness (plain C client of the ABI)."""
import os
import struct
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "cpp", "bin", "abi_harness")


def write_inputs(tmp, rules, arena, offs):
    rp, qp = os.path.join(tmp, "rules.txt"), os.path.join(tmp, "requests.bin")
    with open(rp, "w") as f:
        for r in rules:
            f.write("\t".join([r.Path, r.Method, r.Host, "\x1f".join(r.Headers)]) + "\n")
    with open(qp, "wb") as f:
        f.write(struct.pack("<QQ", len(offs), arena.nbytes))
        f.write(np.ascontiguousarray(offs, dtype=np.uint64).tobytes())
        f.write(np.ascontiguousarray(arena, dtype=np.uint8).tobytes())
    return rp, qp


def run(tmp, rules, arena, offs, threads, iters, timeout=240, batcher=False):
    rp, qp = write_inputs(tmp, rules, arena, offs)
    out = os.path.join(tmp, "out.bin")
    p = subprocess.run([HARNESS, rp, qp, str(threads), str(iters), out] + (["batcher"] if batcher else []),
                       capture_output=True, text=True, timeout=timeout)
    res = None
    if os.path.exists(out):
        raw = open(out, "rb").read()
        n = len(offs)
        res = (np.frombuffer(raw[:4 * n], dtype=np.int32), np.frombuffer(raw[4 * n:], dtype=np.uint64))
    return p, res
