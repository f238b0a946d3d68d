#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per kernel, consecutive runs of
launches (one run per bench workload, in launch order) with mean/min/max
duration, so the render-kernel average can be compared with bench.py's
in-stream HIP-event mean for the same workload.

  python scripts/prof_summary.py gpurun_out/prof_r1/bench_kernel_trace.csv [--labels a,b]
"""
import csv
import json
import sys


def main():
    path = sys.argv[1]
    labels = []
    if "--labels" in sys.argv:
        labels = sys.argv[sys.argv.index("--labels") + 1].split(",")
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    runs = []
    for r in rows:
        name = r["Kernel_Name"]
        if "render_" not in name:
            continue
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        key = (name, r["Grid_Size_X"], r["Grid_Size_Y"], r["LDS_Block_Size"])
        # a new run starts when the launch shape changes or after a long idle gap
        start = int(r["Start_Timestamp"])
        if runs and runs[-1]["key"] == key and start - runs[-1]["last_end"] < 50e6:
            runs[-1]["ms"].append(dur)
            runs[-1]["last_end"] = int(r["End_Timestamp"])
        else:
            runs.append({"key": key, "ms": [dur], "last_end": int(r["End_Timestamp"]),
                         "vgpr": r.get("VGPR_Count"), "sgpr": r.get("SGPR_Count"),
                         "scratch": r.get("Scratch_Size"), "lds": r["LDS_Block_Size"]})
    out = []
    for i, run in enumerate(runs):
        ms = run["ms"]
        out.append({"label": labels[i] if i < len(labels) else f"run{i}", "kernel": run["key"][0][:60],
                    "grid": [int(run["key"][1]), int(run["key"][2])], "launches": len(ms),
                    "mean_ms": round(sum(ms) / len(ms), 4), "min_ms": round(min(ms), 4),
                    "max_ms": round(max(ms), 4), "vgpr": run["vgpr"], "sgpr": run["sgpr"],
                    "scratch": run["scratch"], "lds_bytes": run["lds"]})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
