#!/usr/bin/env python3
"""One line per bench JSON found in the given files: config, ms/step, kernel ms, roofline frac."""
import json
import sys

for f in sys.argv[1:]:
    try:
        lines = open(f).read().splitlines()
    except OSError as e:
        print(f, "missing", e)
        continue
    for l in lines:
        if l.startswith("{"):
            d = json.loads(l)
            r = d.get("roofline", {})
            print(f"{f}: {d['config'].get('workload')} ms/step {d['ms_per_step']:.3f} kernel {r.get('kernel_ms', 0):.3f} "
                  f"frac {r.get('frac', 0):.3f} value {d['value']:.4g} counters_ok {d.get('counters_ok')}")
