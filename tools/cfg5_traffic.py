#!/usr/bin/env python3
"""Config 5: which record bytes the HTTP kernel actually fetches (CPU estimate,
explains profiles' FETCH_SIZE well below the algorithmic bytes).

The kernel stages a tile of consecutive records whose window fits the wave's
8 KiB stage (coalesced copy: every byte fetched); a record that does not fit
(> 8 KiB: the 1-64 KiB x-blob values) is read from HBM directly, and only the
bytes its walks touch are fetched: the fixed header, the header directory,
method / path / authority, header names, and the first bytes of the x-blob
value (its literal-trie walk dies within a few bytes for random values).
Tiles are simulated as one sequential stream (the kernel's per-wave shares
cut it at ~16k more places, a negligible difference)."""
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cilium_amd import workloads as W  # noqa: E402

STAGE = 8192
LINE = 128


def main(n=1_000_000):
    arena, offs = W.requests(5, 0, n, n_rules=100_000, threads=8)
    tot = arena.nbytes - 64
    o = offs.astype(np.int64)
    sizes = np.diff(np.append(o, tot))
    staged, direct, i = 0, [], 0
    while i < n:
        base = o[i] & ~15
        k = 0
        while k < 64 and i + k < n and (o[i + k] + sizes[i + k]) - base <= STAGE:
            k += 1
        if k == 0:
            direct.append(i)
            i += 1
            continue
        staged += (o[i + k - 1] + sizes[i + k - 1]) - base
        i += k
    buf = arena.tobytes()
    touched = 0
    for r in direct:
        off = int(o[r])
        w = struct.unpack_from("<5I", buf, off)
        nh, ml, pl, al = w[2] >> 24, w[3] & 0xFFFF, w[3] >> 16, w[4] & 0xFFFF
        front = 20 + 4 * nh + ml + pl + al
        for j in range(nh):
            e = struct.unpack_from("<I", buf, off + 20 + 4 * j)[0]
            nl, vl = e & 0xFFFF, e >> 16
            front += nl + (vl if vl <= 64 else 16)
        touched += ((front + LINE - 1) // LINE + 1) * LINE  # + the blob value's first line
    print(f"{n} requests: algorithmic record bytes {tot / 1e9:.3f} GB")
    print(f"  staged tiles: {staged / 1e9:.3f} GB fetched in full")
    print(f"  {len(direct)} records larger than the stage: {sizes[direct].sum() / 1e9:.3f} GB, "
          f"~{touched / 1e9:.4f} GB of it touched by the walks")
    print(f"  record bytes fetched ~{(staged + touched) / 1e9:.3f} GB "
          f"({(staged + touched) / tot:.2f} x algorithmic); + offsets {8 * n / 1e9:.3f} GB, verdicts {4 * n / 1e9:.3f} GB")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000)
