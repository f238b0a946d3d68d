#!/usr/bin/env python3
"""Per-wave timeline of ONE multi-frame launch (the bench's launch shape), from
a -DRT_STAMPS build (RT_HIP_LIB) with RT_HIP_STAMPS_FILE set: renders F frames
of the scene's camera per launch a few times, then summarises the last
launch's waves: span, when the resident-wave count falls, and the waves that
end last (group slot, frame, start, duration).
  RT_HIP_LIB=build_variants/librt_hip_stamps.so RT_HIP_STAMPS_FILE=/tmp/tl.bin \\
      python scripts/timeline_frames.py synth200 1920 1080 4 16"""
import os
import sys

import numpy as np

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
for _ in range(3):
    r.render_frames_async([sc.camera()] * F, W, H, D, None, buf.data_ptr(), H * W * 3)
    st = r.stats()
print("launch kernel ms (render + deferred):", r.kernel_times(8)[-1:])
a = np.fromfile(os.environ["RT_HIP_STAMPS_FILE"], dtype=np.uint64).reshape(-1, 16)
n = int((a[:, 1] > 0).sum())
a = a[: max(i for i in range(len(a)) if a[i, 1] > 0) + 1]
s0 = a[:, 0].astype(np.float64)
ok = a[:, 1] > 0
t0 = s0[ok].min()
s = (s0 - t0) / 100.0
e = (a[:, 1].astype(np.float64) - t0) / 100.0
d = e - s
s, e, d = s[ok], e[ok], d[ok]
ids = np.nonzero(ok)[0]
print(f"waves {n}  span {e.max():.1f} us  dur mean {d.mean():.1f} med {np.median(d):.1f} p99 {np.percentile(d, 99):.1f} "
      f"max {d.max():.1f} us")
for q in (50, 90, 99, 99.9, 100):
    print(f"  {q}% of waves started by {np.percentile(s, q):.1f} us, ended by {np.percentile(e, q):.1f} us")
ts = np.linspace(0, e.max(), 41)
print("  resident waves over time:", " ".join(str(int(((s <= t) & (e > t)).sum())) for t in ts))
order = np.argsort(-e)[:20]
print("  last-ending waves: workgroup (group slot, frame) start dur end (us)")
for w in order:
    b = int(ids[w])
    print(f"   {b:7d} ({b // F:5d}, {b % F:2d}) {s[w]:8.1f} {d[w]:7.1f} {e[w]:8.1f}")
longest = np.argsort(-d)[:10]
print("  longest waves: workgroup (group slot, frame) start dur end (us)")
for w in longest:
    b = int(ids[w])
    print(f"   {b:7d} ({b // F:5d}, {b % F:2d}) {s[w]:8.1f} {d[w]:7.1f} {e[w]:8.1f}")
grp = ids // F
for lo, hi in ((0, 100), (100, 500), (500, 2000), (2000, 8100)):
    m = (grp >= lo) & (grp < hi)
    if m.any():
        print(f"  groups {lo}-{hi}: waves {m.sum()} dur mean {d[m].mean():.1f} max {d[m].max():.1f} us, "
              f"start max {s[m].max():.1f} us")
