#!/usr/bin/env python3
"""Mean per-dispatch PMC values of the render kernel from gpu_pmc.sh output dirs."""
import collections, csv, glob, json, sys
base = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "render_kernel"
out = {}
for f in sorted(glob.glob(f"{base}/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        out[k] = sum(v) / len(v)
print(json.dumps(out, indent=1))
