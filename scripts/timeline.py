#!/usr/bin/env python3
"""Render a workload a few times with the diagnostic library (RT_HIP_LIB pointing
at a -DRT_STAMPS build, RT_HIP_STAMPS_FILE set) so the last frame's per-wave
timeline is dumped; then summarise it (run with --analyse FILE here)."""
import os
import sys

if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
    import numpy as np
    a = np.fromfile(sys.argv[2], dtype=np.uint64).reshape(-1, 16)
    n = int(sys.argv[3]) if len(sys.argv) > 3 else (a[:, 1] > 0).sum()
    a = a[:n]
    t0 = a[:, 0].min()
    s = (a[:, 0] - t0) / 100.0  # us (100 MHz)
    e = (a[:, 1] - t0) / 100.0
    d = e - s
    print(f"waves {n}  span {e.max():.1f} us  dur mean {d.mean():.1f} med {np.median(d):.1f} p99 {np.percentile(d,99):.1f} max {d.max():.1f} us")
    for q in (0.5, 0.9, 0.99, 1.0):
        print(f"  {q*100:.0f}% of waves started by {np.percentile(s, q*100):.1f} us, ended by {np.percentile(e, q*100):.1f} us")
    # concurrency over time
    ts = np.linspace(0, e.max(), 41)
    conc = [((s <= t) & (e > t)).sum() for t in ts]
    print("  resident waves over time:", " ".join(str(c) for c in conc))
    xcc = (a[:, 2] >> 32) & 0xF
    print("  waves per XCC:", np.bincount(xcc.astype(np.int64), minlength=8).tolist())
    # duration by tile row (image y)
    W_tiles = int(sys.argv[4]) if len(sys.argv) > 4 else 240
    rows = np.arange(n) // W_tiles
    per_row = [d[rows == r].mean() for r in range(rows.max() + 1)]
    print("  mean wave duration per tile row (us):", " ".join(f"{x:.0f}" for x in per_row))
    order = np.argsort(-d)[:12]
    print("  slowest waves: id(tile x,y) dur_us | cycles: bound cull cand shade bvh total | iters sweeps")
    for w in order:
        it, sw = int(a[w, 8]) & 0xFFFFFFFF, int(a[w, 8]) >> 32
        print(f"   {w:6d} ({w % W_tiles:3d},{w // W_tiles:3d}) {d[w]:7.1f} bvhmax {a[w,9]:5d} | {a[w,3]:8d} {a[w,4]:8d} {a[w,5]:9d} {a[w,6]:8d} {a[w,10]:8d} {a[w,7]:9d} | {it:5d} {sw:4d}")
    print("  slowest waves: closest-sweep shadow-sweep bvh cycles | bvh wave trips, max lane steps")
    for w in order:
        print(f"   {w:6d} {a[w,12]:9d} {a[w,13]:9d} {a[w,10]:9d} | {a[w,14]:6d} {a[w,9]:6d}")
    med = np.argsort(d)[len(d)//2]
    w = med
    print(f"  median wave {w}: {d[w]:.1f} us | {a[w,3]} {a[w,4]} {a[w,5]} {a[w,6]} {a[w,10]} {a[w,7]} | {int(a[w,8]) & 0xFFFFFFFF} {int(a[w,8]) >> 32}")
    sys.exit(0)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs420-ray-tracer_amd"))
import rt_hip  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "synth200"
W, H, D = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 4)
sc = rt_hip.Scene.load(os.path.join(REPO, "cs420-ray-tracer_amd", "scenes", scene + ".txt"))
r = rt_hip.Renderer(0)
r.upload(sc)
# SHARD=r/G renders rank r's cyclic 8-row bands of G (the N = G bench's per-rank launch)
shard = os.environ.get("SHARD")
rows = rt_hip.rows_for_shard(H, 8, *(int(x) for x in shard.split("/"))) if shard else None
for _ in range(4):
    _, st = r.render(sc.camera(), W, H, D, rows)
print("kernel ms", st.kernel_ms)
