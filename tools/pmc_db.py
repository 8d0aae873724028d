"""Average PMC counters per dispatch of the l7m kernels from a rocprofv3
results database (rocpd sqlite, the default output format)."""
import collections
import glob
import sqlite3
import sys

for db in sys.argv[1:] or sorted(glob.glob("**/*_results.db", recursive=True)):
    c = sqlite3.connect(db)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    geo = {}
    for name, did, cname, val, grid, wg, vgpr, sgpr, lds, dur in c.execute(
            "select kernel_name, dispatch_id, counter_name, value, grid_size, workgroup_size, vgpr_count, "
            "sgpr_count, lds_block_size, duration from counters_collection"):
        if "l7m" not in name:
            continue
        key = name.split("(")[0][-70:]
        agg[key][cname] += val
        disp[key].add((did, dur))
        geo[key] = (grid, wg, vgpr, sgpr, lds)
    for k, d in agg.items():
        nd = len(disp[k])
        grid, wg, vgpr, sgpr, lds = geo[k]
        print(db, k, f"dispatches={nd} grid={grid} wg={wg} vgpr={vgpr} sgpr={sgpr} lds={lds}")
        for cn, v in sorted(d.items()):
            print(f"    {cn:28s} {v / nd:.6g}")
