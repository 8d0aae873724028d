"""Average PMC counters per dispatch of the l7m kernels (rocprofv3 csv)."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "."
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    disp = collections.defaultdict(set)
    geo = {}
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "l7m" not in name:
            continue
        m = re.search(r"(\w+_kernel)", name)
        key = m.group(1) if m else name[:60]
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        disp[key].add(r["Dispatch_Id"])
        geo[key] = (r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"], r["SGPR_Count"])
    for k, d in agg.items():
        grid, wg, lds, vgpr, sgpr = geo[k]
        nd = len(disp[k])
        vals = {c: sum(v) / nd for c, v in d.items()}
        print(f.split("/")[-2], k, f"dispatches={nd} grid={grid} wg={wg} lds={lds} vgpr={vgpr} sgpr={sgpr}")
        for c, v in sorted(vals.items()):
            print(f"    {c:28s} {v:.6g}")
