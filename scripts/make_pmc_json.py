#!/usr/bin/env python3
"""Fold scripts/gpu_profile.sh counter passes into profiles/pmc_traffic.json (read by bench.py).

  python scripts/make_pmc_json.py WORKLOAD PMC_DIR [KERNEL_SUBSTR]

Per FRAME: every counter is summed over the multi-frame render dispatches
(the largest render grid of the run; FRAMES frames each, bench.py's
--frames-per-launch, default 32) -- each with the render_deferred dispatch
that follows it (the launch's deep reflection rays) -- and divided by the
frames they rendered:
  hbm_bytes_per_frame = (2 * FETCH_SIZE + WRITE_SIZE) * 1024  (rocprofv3 reports
      KiB; FETCH_SIZE doubled: MI355X_MICROARCH.md's gfx950 correction -- it
      reports half the bytes of 128-B requests; fetch_bytes / write_bytes are
      the raw per-frame values)
  fp64_share_of_valu_insts = (ADD + MUL + FMA + TRANS)_F64 / SQ_INSTS_VALU
  valu_lane_utilization = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)
      (rocprofv3's VALUUtilization: the mean fraction of a wave's lanes active
      per VALU cycle)
  kernel_src_sha = bench.kernel_source_sha() of the tree the passes ran on
  valu_busy = SQ_ACTIVE_INST_VALU * 4 / (SIMDs * GRBM_GUI_ACTIVE / XCDs)
  fp64_flops_per_frame = 64 * (ADD + MUL + 2 FMA + TRANS)_F64 wave-instructions
      (an upper bound: it assumes every lane of the wave is active)
"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS, XCDS = 1024, 8
FRAMES = int(os.environ.get("FRAMES", "32"))  # frames per multi-frame launch of the PMC runs (bench.py's default)


def main():
    workload, base = sys.argv[1], sys.argv[2]
    kern = sys.argv[3] if len(sys.argv) > 3 else "render_"
    vals = {}
    for f in sorted(glob.glob(f"{base}/p*/run_counter_collection.csv")):
        rows = [r for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        main = [r for r in rows if "render_deferred" not in r["Kernel_Name"]]
        if not main:
            continue
        # the multi-frame launches only (the largest render grid; bench.py's
        # one-frame ray-count launch has the one-frame kernel split), each with
        # the render_deferred dispatch that follows it (its deep reflection rays)
        gmax = max(int(r["Grid_Size"]) for r in main)
        last_main_grid, keep = None, set()
        for r in sorted({(int(r["Dispatch_Id"]), r["Kernel_Name"], int(r["Grid_Size"])) for r in rows}):
            did, name, grid = r
            if "render_deferred" not in name:
                last_main_grid = grid
            if last_main_grid == gmax:
                keep.add(did)
        agg = collections.defaultdict(float)
        frames = collections.defaultdict(float)
        for r in rows:
            if int(r["Dispatch_Id"]) not in keep:
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            if "render_deferred" not in r["Kernel_Name"]:
                frames[r["Counter_Name"]] += FRAMES
        for k, v in agg.items():
            vals[k] = v / frames[k]
    out = {}
    if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
        out["fetch_bytes"] = round(vals["FETCH_SIZE"] * 1024)
        out["write_bytes"] = round(vals["WRITE_SIZE"] * 1024)
        out["hbm_bytes_per_frame"] = 2 * out["fetch_bytes"] + out["write_bytes"]
    if "SQ_ACTIVE_INST_VALU" in vals and "GRBM_GUI_ACTIVE" in vals:
        cycles = vals["GRBM_GUI_ACTIVE"] / XCDS
        out["kernel_cycles_per_frame"] = round(cycles)
        out["valu_busy"] = round(vals["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * cycles), 4)
    f64 = [vals.get("SQ_INSTS_VALU_%s_F64" % k) for k in ("ADD", "MUL", "FMA", "TRANS")]
    if None not in f64:
        out["fp64_flops_per_frame"] = round(64 * (f64[0] + f64[1] + 2 * f64[2] + f64[3]))
        out["valu_insts_per_frame"] = round(vals.get("SQ_INSTS_VALU", 0))
        if vals.get("SQ_INSTS_VALU"):
            out["fp64_share_of_valu_insts"] = round(sum(f64) / vals["SQ_INSTS_VALU"], 4)
    if vals.get("SQ_THREAD_CYCLES_VALU") and vals.get("SQ_ACTIVE_INST_VALU"):
        out["valu_lane_utilization"] = round(vals["SQ_THREAD_CYCLES_VALU"] / (64 * vals["SQ_ACTIVE_INST_VALU"]), 4)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench  # noqa: E402  (the source hash bench.py checks)

    # the hash of the kernel sources the passes ran on: gpu_profile.sh records it
    # beside them (kernel_src_sha.txt); else the tree this runs in
    rec = [os.path.join(base, q, "kernel_src_sha.txt") for q in (".", "..", "../..")]
    rec = [q for q in rec if os.path.exists(q)]
    out["kernel_src_sha"] = open(rec[0]).read().strip() if rec else bench.kernel_source_sha()
    out["source"] = os.path.relpath(base, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    out["counters"] = {k: round(v, 1) for k, v in sorted(vals.items())}
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    data[workload] = out
    with open(path, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    print(json.dumps({workload: {k: v for k, v in out.items() if k != "counters"}}))


if __name__ == "__main__":
    main()
