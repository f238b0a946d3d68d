#!/usr/bin/env python3
"""Per-frame kernel time of a workload at several depths, 16 frames per launch:
the cost of each reflection level.  depth_time.py scene W H d1 d2 ..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs420-ray-tracer_amd"))
import torch  # noqa: E402
import rt_hip  # noqa: E402

scene, W, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
sc = rt_hip.Scene.load(os.path.join(REPO, "cs420-ray-tracer_amd", "scenes", scene + ".txt"))
r = rt_hip.Renderer(0)
r.upload(sc)
F = 16
out = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda:0")
for d in map(int, sys.argv[4:]):
    _, st = r.render(sc.camera(), W, H, d)
    for _ in range(2):
        r.render_frames_async([sc.camera()] * F, W, H, d, None, out.data_ptr(), H * W * 3)
    r.kernel_times()
    for _ in range(6):
        r.render_frames_async([sc.camera()] * F, W, H, d, None, out.data_ptr(), H * W * 3)
    kt = r.kernel_times()
    print(d, st.rays_primary, st.rays_shadow, st.rays_reflect, "%.4f ms/frame" % (sum(kt) / len(kt) / F), flush=True)
