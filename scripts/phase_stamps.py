#!/usr/bin/env python3
"""Per-phase cycle counts of the render kernels (a -DRT_STAMPS build): F
frames of a workload in one launch, a few times; the library prints cycles per
wave per phase (closest hits, shadow queries, per-light setup, shading, whole
wave) for the last launch.  The stamps drain memory before each reading, so
the totals are slower than the product's; the shares are what they are for.
  make -C cs420-ray-tracer_amd/csrc variant NAME=stamps DEFS=-DRT_STAMPS
  RT_HIP_LIB=build_variants/librt_hip_stamps.so RT_HIP_STAMPS=1 \\
      python scripts/phase_stamps.py synth200 1920 1080 4 16"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs420-ray-tracer_amd"))
import torch  # noqa: E402
import rt_hip  # noqa: E402

scene = sys.argv[1]
W, H, D, F = (int(v) for v in sys.argv[2:6])
sc = rt_hip.Scene.load(os.path.join(REPO, "cs420-ray-tracer_amd", "scenes", scene + ".txt"))
r = rt_hip.Renderer(0)
r.upload(sc)
buf = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda:0")
for k in range(3):
    if k == 2:
        print(f"--- {scene} {W}x{H} d{D}, {F} frames per launch", file=sys.stderr, flush=True)
    r.render_frames_async([sc.camera()] * F, W, H, D, None, buf.data_ptr(), H * W * 3)
    st = r.stats() if k == 2 else None
    if k < 2:
        torch.cuda.synchronize()
print("kernel ms per frame", r.kernel_times(8)[-1] / F, "rays", st.rays, file=sys.stderr)
