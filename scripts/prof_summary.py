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
    current = {}  # launch shape -> its open run (render_kernel and render_deferred interleave)
    for r in rows:
        name = r["Kernel_Name"]
        if "render_" not in name:
            continue
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        key = (name, r["Grid_Size_X"], r["Grid_Size_Y"], r["LDS_Block_Size"])
        # a new run of a shape starts after a long idle gap since its previous launch
        start = int(r["Start_Timestamp"])
        run = current.get(key)
        if run is not None and start - run["last_end"] < 50e6:
            run["ms"].append(dur)
            run["last_end"] = int(r["End_Timestamp"])
        else:
            run = {"key": key, "ms": [dur], "last_end": int(r["End_Timestamp"]),
                   "vgpr": r.get("VGPR_Count"), "sgpr": r.get("SGPR_Count"),
                   "scratch": r.get("Scratch_Size"), "lds": r["LDS_Block_Size"]}
            runs.append(run)
            current[key] = run
    out = []
    for i, run in enumerate(runs):
        ms = run["ms"]
        out.append({"label": labels[i] if i < len(labels) else f"run{i}", "kernel": run["key"][0][:60],
                    "grid": [int(run["key"][1]), int(run["key"][2])], "launches": len(ms),
                    "mean_ms": round(sum(ms) / len(ms), 4),
                    # the bench times the launches after its warm-up one
                    "mean_ms_after_first": round(sum(ms[1:]) / len(ms[1:]), 4) if len(ms) > 1 else None,
                    "min_ms": round(min(ms), 4),
                    "max_ms": round(max(ms), 4), "vgpr": run["vgpr"], "sgpr": run["sgpr"],
                    "scratch": run["scratch"], "lds_bytes": run["lds"]})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
