"""Per-rank kernel time of a row-sharded frame, measured on ONE GPU: for G in
(1, 2, 4, 8) every shard r of G is rendered back to back and timed with the
library's in-stream events.  max over r of the shard time is what rank r's
kernel costs in the N = G bench, so G * max / full-frame time is the strong
scaling loss that comes from the kernel itself (tail + launch granularity),
before any RCCL cost.

usage: python scripts/shard_probe.py [workload] [frames]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs420-ray-tracer_amd"))
import torch  # noqa: E402  (torch's HIP runtime first)
import rt_hip  # noqa: E402

WORK = {"synth200_1920x1080_d4": ("synth200", 1920, 1080, 4), "complex_1920x1080_d4": ("complex", 1920, 1080, 4),
        "complex_3840x2160_d4": ("complex", 3840, 2160, 4), "synth10k_3840x2160_d6": ("synth10k", 3840, 2160, 6)}
wl = sys.argv[1] if len(sys.argv) > 1 else "synth200_1920x1080_d4"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 30
band = int(os.environ.get("BAND", "8"))
fpl = int(os.environ.get("FPL", "1"))  # frames per launch (rt_render_frames_async); times are per frame
name, W, H, D = WORK[wl]
scene = rt_hip.Scene.load(os.path.join(ROOT, "cs420-ray-tracer_amd", "scenes", name + ".txt"))
cam = scene.camera()
# PROBE_VARIANT=tuning: the tuning build, so its RT_HIP_* knobs apply
r = rt_hip.Renderer(0, variant=os.environ.get("PROBE_VARIANT") or None)
r.upload(scene)
out = torch.empty((fpl, H, W, 3), dtype=torch.uint8, device="cuda:0")
res = {"workload": wl, "band": band, "frames_per_launch": fpl}


def launch(rows):
    if fpl == 1:
        r.render_async(cam, W, H, D, rows, out.data_ptr())
    else:
        r.render_frames_async([cam] * fpl, W, H, D, rows, out.data_ptr(), rows.count * W * 3)


GS = tuple(int(g) for g in os.environ.get("GS", "1,2,4,8").split(","))
for G in GS:
    per = []
    for k in range(G):
        rows = rt_hip.rows_for_shard(H, band, k, G) if G > 1 else rt_hip.rt_rows(1, 0, 1, H)
        for _ in range(3):
            launch(rows)
        r.kernel_times()
        for _ in range(frames):
            launch(rows)
        kt = r.kernel_times(frames)
        per.append(sum(kt) / len(kt) / fpl)
    res[f"G{G}"] = {"max_ms": round(max(per), 4), "mean_ms": round(sum(per) / G, 4),
                    "shard_ms": [round(x, 4) for x in per]}
if "G1" in res:
    full = res["G1"]["max_ms"]
    for G in GS:
        if G > 1:
            res[f"G{G}"]["kernel_eff"] = round(full / (G * res[f"G{G}"]["max_ms"]), 3)
print(json.dumps(res))
r.close()
