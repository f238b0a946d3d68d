#!/usr/bin/env python3
"""Render one workload at several depths (one launch each, after a warm-up),
for per-level PMC attribution under rocprofv3:  depth_probe.py scene W H d1 d2 ..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs420-ray-tracer_amd"))
import rt_hip  # noqa: E402

scene, W, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
sc = rt_hip.Scene.load(os.path.join(REPO, "cs420-ray-tracer_amd", "scenes", scene + ".txt"))
r = rt_hip.Renderer(0)
r.upload(sc)
for d in map(int, sys.argv[4:]):
    r.render(sc.camera(), W, H, d)
    _, st = r.render(sc.camera(), W, H, d)
    print(d, st.rays_primary, st.rays_shadow, st.rays_reflect, st.kernel_ms, flush=True)
