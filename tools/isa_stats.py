#!/usr/bin/env python3
"""Static ISA summary of the kernels in one .hip file (gfx950), for A/B work
on code generation without a GPU:

    tools/isa_stats.py cilium_amd/csrc/l7m_kafka.hip [-DFLAG ...] [-k substr]

Prints per kernel: VGPR / SGPR / LDS / scratch from the code object metadata
and instruction counts by class (VALU, SALU, DS, global, branches, waitcnt).
"""
import argparse
import os
import re
import subprocess
import tempfile

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("-k", "--kernel", default="", help="substring of the kernel symbol")
ap.add_argument("flags", nargs="*")
a, extra = ap.parse_known_args()
flags = a.flags + extra

with tempfile.TemporaryDirectory() as td:
    asm = os.path.join(td, "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-munsafe-fp-atomics", *flags, a.src, "-o", asm], check=True)
    text = open(asm).read()

funcs = {}
cur = None
for line in text.splitlines():
    m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
    if m:
        cur = m.group(1)
        funcs[cur] = []
        continue
    if cur and line.startswith("\t.end_amdhsa_kernel"):
        cur = None
    if cur and line.startswith("\t") and not line.startswith("\t."):
        funcs[cur].append(line.strip())

meta = {}
for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", text, re.S):
    body = m.group(2)
    g = lambda k: (re.search(r"\.%s (\d+)" % k, body) or [None, "?"])[1]
    meta[m.group(1)] = (g("amdhsa_next_free_vgpr"), g("amdhsa_next_free_sgpr"),
                        g("amdhsa_group_segment_fixed_size"), g("amdhsa_private_segment_fixed_size"))

for name, ins in funcs.items():
    if a.kernel not in name or name not in meta:
        continue
    c = dict(valu=0, salu=0, ds=0, glob=0, br=0, wait=0)
    for i in ins:
        op = i.split()[0] if i else ""
        if op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("s_waitcnt"):
            c["wait"] += 1
        elif op.startswith("s_cbranch") or op.startswith("s_branch"):
            c["br"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith("ds_"):
            c["ds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["glob"] += 1
    v, s, l, p = meta[name]
    print(f"{name[:90]}\n   vgpr {v} sgpr {s} lds {l} scratch {p} | lines {len(ins)} " +
          " ".join(f"{k} {n}" for k, n in c.items()))
