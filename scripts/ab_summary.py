#!/usr/bin/env python3
"""One line per bench JSON (the A/B runs of scripts/gpu_libab.sh): the headline
ms/frame, the single-frame kernel / wall ms, the moving-camera ms/frame and
the also-line.   python scripts/ab_summary.py gpurun_out/r4f/ab_*.json"""
import json
import sys

for p in sys.argv[1:]:
    lines = [l for l in open(p).read().splitlines() if l.startswith("{")]
    if not lines:
        print(p, "no JSON line")
        continue
    d = json.loads(lines[-1])
    sf, mc = d.get("single_frame") or {}, d.get("moving_camera") or {}
    also = {k: v.get("ms_per_step") for k, v in (d.get("also") or {}).items()}
    print(f"{p.split('/')[-1]:34s} ms/frame {d['ms_per_step']:.4f}  single k {sf.get('kernel_ms')} wall {sf.get('wall_ms')}"
          f"  moving {mc.get('kernel_ms_per_frame')}  also {also}")
