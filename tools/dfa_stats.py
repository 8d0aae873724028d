"""Print the packed-DFA footprint of the benchmark rule sets (dev tool)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from cilium_amd import l7match as L  # noqa: E402
from cilium_amd import workloads as W  # noqa: E402
from program_interp import HttpProgram  # noqa: E402

KNONE = 0xFFFFFFFF


def main():
    for cfg, n in ((1, None), (2, None), (2, 5000)):
        rules = W.rules(cfg, n_rules=n) if n else W.rules(cfg)
        t = time.time()
        rs = L.RuleSet.compile_http(rules)
        dt = time.time() - t
        P = HttpProgram(rs.program())
        print(f"config {cfg}: {len(rules)} rules, compile {dt:.2f} s, program {rs.info.program_bytes / 1024:.0f} KiB, "
              f"LDS image {P.h['lds_image_words'] * 4 / 1024:.1f} KiB")
        for d in P.dfas:
            name = "names" if d["field"] == KNONE else f"field {d['field']}"
            print(f"   {name:9s} slots {d['n_slots']:6d} states {d['nstates']:6d} region {d['region']:6d} "
                  f"lds {d['lds_table'] != KNONE} ct_lds {d['lds_ct'] != KNONE}")


if __name__ == "__main__":
    main()
