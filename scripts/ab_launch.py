"""A/B of launch-shape knobs on one GPU (a tuning tool, not a test): for each
setting (RT_HIP_* environment read at rt_create), per workload:
  single-frame launches from fresh camera positions (kernel ms, median),
  the batched rate (launches of F frames, kernel ms per frame),
and a byte check that every setting renders the same image.
  python scripts/ab_launch.py VAR=v1,v2,... [workload ...]
  python scripts/ab_launch.py "A=1+B=0;A=2;default" [workload ...]   (settings of several knobs)
Every setting runs on the tuning build (variants/librt_hip_tuning.so), the
default one included, so the A/B compares one library -- or on the library
RT_HIP_LIB names, when set (scripts/ab_libs.sh)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs420-ray-tracer_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
import rt_hip  # noqa: E402


def run(workload, env, reps=3):
    name, W, H, D = bench.WORKLOADS[workload]
    for k, v in env.items():
        os.environ[k] = v
    try:
        sc = rt_hip.Scene.load(os.path.join(bench.PKG, "scenes", name + ".txt"))
        cam = sc.camera()
        # the tuning build, unless RT_HIP_LIB names a library (scripts/ab_libs.sh's A/B of builds)
        r = rt_hip.Renderer(0, variant=None if os.environ.get("RT_HIP_LIB") else "tuning")
        r.upload(sc)
        info = bench.info_or_none(r)
        rows = rt_hip.rt_rows(1, 0, 1, H)
        F = 32
        buf = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda:0")
        one = bench.single_frame(rt_hip, r, cam, W, H, D, rows, buf[0].data_ptr(), samples=7)
        res = {"single_ms": one["kernel_ms"], "single_wall": one["wall_ms"]}
        if info is not None:
            res.update(upload_ms=round(info.upload_ms, 2), sphere_grids=info.sphere_grids,
                       sg_entries=info.sphere_grid_entries, sg_build_ms=round(info.sphere_grid_build_ms, 2))
        for nf in (32, 20, 8):
            cams = [cam] * nf
            r.render_frames_async(cams, W, H, D, rows, buf.data_ptr(), H * W * 3)
            r.stats()
            r.kernel_times()
            for _ in range(reps):
                r.render_frames_async(cams, W, H, D, rows, buf.data_ptr(), H * W * 3)
            kt = r.kernel_times(reps)
            res[f"f{nf}_ms_per_frame"] = round(min(kt) / nf, 4)
        r.render_async(cam, W, H, D, rows, buf[0].data_ptr())
        r.stats()
        img = bytes(buf[0].cpu().numpy().tobytes())
        r.close()
        return res, img
    finally:
        for k in env:
            del os.environ[k]


def settings(arg):
    if ";" in arg or "+" in arg:  # "A=1+B=0;A=2;default"
        out = []
        for setting in arg.split(";"):
            out.append({} if setting == "default" else dict(kv.split("=", 1) for kv in setting.split("+")))
        return out
    var, vals = arg.split("=")
    return [{} if v == "default" else {var: v} for v in vals.split(",")]


def main():
    loads = sys.argv[2:] or ["synth200_1920x1080_d4", "complex_1920x1080_d4"]
    for wl in loads:
        ref = None
        for env in settings(sys.argv[1]):
            res, img = run(wl, env)
            same = ref is None or img == ref
            ref = ref or img
            print(f"{wl} {env or 'default'}: {res} same_image={same}", flush=True)
            assert same


if __name__ == "__main__":
    main()
