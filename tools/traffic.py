"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of a bench run into the
per-launch HBM traffic of the l7m kernel (bench.py's roofline.traffic).

    python tools/traffic.py <pmc_FETCH_SIZE dir> <pmc_WRITE_SIZE dir> <config> <out.json>

FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes
of a wide coalesced stream (MI355X_MICROARCH.md §HBM), so
traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes.  The .so hash ties the
number to the kernel build it was measured on."""
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "l7m" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return sorted(vals.values())


def so_hash():
    with open(os.path.join(ROOT, "cilium_amd", "libl7match.so"), "rb") as f:
        return hashlib.md5(f.read()).hexdigest()


def main():
    fdir, wdir, cfg, out = sys.argv[1:5]
    fetch = per_dispatch(fdir, "FETCH_SIZE")
    write = per_dispatch(wdir, "WRITE_SIZE")
    assert fetch and write, "no l7m dispatches found"
    kib_f = max(fetch)  # the timed launch (largest dispatch)
    kib_w = max(write)
    sys.path.insert(0, ROOT)
    from cilium_amd.codehash import code_md5, kernel_md5
    res = {"config": int(cfg), "fetch_kib": kib_f, "write_kib": kib_w,
           "traffic_bytes": (2 * kib_f + kib_w) * 1024, "so_md5": so_hash(),
           "kernel_md5": kernel_md5(os.path.join(ROOT, "cilium_amd", "libl7match.so")),
           "code_md5": code_md5(os.path.join(ROOT, "cilium_amd", "libl7match.so")),
           "correction": "2 x FETCH_SIZE (gfx950 half-count on wide streams) + WRITE_SIZE, KiB -> bytes"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
