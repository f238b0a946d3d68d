#!/usr/bin/env python3
"""Is a launch that follows an idle GPU slower?  For each idle gap (host sleep
after torch.cuda.synchronize()) and launch shape: a warm launch of WARM frames,
synchronize, sleep, then one launch of F frames; in-stream kernel ms of that
launch per frame (median of REPS).  The bench's timed launch follows a barrier
+ synchronize, i.e. a short idle gap.
  python scripts/idle_gap.py [workload]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs420-ray-tracer_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
import rt_hip  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "synth200_1920x1080_d4"
name, W, H, D = bench.WORKLOADS[wl]
sc = rt_hip.Scene.load(os.path.join(bench.PKG, "scenes", name + ".txt"))
cam = sc.camera()
r = rt_hip.Renderer(0)
r.upload(sc)
r.set_stream(torch.cuda.current_stream().cuda_stream)
buf = torch.empty((32, H, W, 3), dtype=torch.uint8, device="cuda:0")
arr = {n: rt_hip.camera_array([cam] * n) for n in (20, 32)}
REPS = 7


def launch(n):
    r.render_frames_async(arr[n], W, H, D, None, buf.data_ptr(), H * W * 3)


for warm, F in ((32, 20), (20, 20), (32, 32)):
    for gap_us in (0, 100, 1000, 20000):
        per = []
        for _ in range(REPS):
            launch(warm)
            torch.cuda.synchronize()
            if gap_us:
                time.sleep(gap_us * 1e-6)
            launch(F)
            torch.cuda.synchronize()
            per.append(r.kernel_times(2)[-1] / F)
        per.sort()
        print(f"{wl} warm {warm} -> {F} frames, idle {gap_us:6d} us: kernel {per[len(per) // 2]:.4f} ms/frame "
              f"(min {per[0]:.4f}, max {per[-1]:.4f})", flush=True)
    # back to back, no synchronize: the steady state
    per = []
    launch(F)
    for _ in range(REPS):
        launch(F)
    torch.cuda.synchronize()
    per = sorted(t / F for t in r.kernel_times(REPS))
    print(f"{wl} {F} frames back to back: kernel {per[len(per) // 2]:.4f} ms/frame (min {per[0]:.4f})", flush=True)
