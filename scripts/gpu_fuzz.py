"""Randomised parity sweep (a design/validation tool, not a test): random
scenes -- whole or fractional shininess (40 % of scenes: int_pow and dd_pow),
1 to 1,500 spheres (so both the cull sweeps and the always-BVH
paths, render_deferred and render_deferred_walk), tiny to huge radii, mirror
clouds, 0 to 6 lights (FUZZ_NEAR_LIGHTS=1: half of them just outside a
sphere), cameras inside spheres -- rendered on cuda:0 through
the C-ABI at small sizes and random depths, against the oracle byte for byte
and ray count for ray count; every third scene is also rendered as three
frames of one launch (rt_render_frames_async: the deferred kernel and, for
scenes with the uniform grid, the XCD frame mapping), each frame against the
same oracle image, and as three frames from three camera positions (a
device-built camera grid per frame when the launch builds grids), each
against the oracle at its camera.  Knobs (RT_HIP_*) apply as set in the environment, e.g.
RT_HIP_BEHIND_GRID=1 RT_HIP_BVH_ALWAYS=1 puts every scene on the uniform
grid.  Prints one line per scene and a summary; exits non-zero on the first
mismatch.
  python scripts/gpu_fuzz.py [SECONDS] [SEED]"""
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs420-ray-tracer_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import torch  # noqa: E402  (torch's HIP runtime first; frame buffers)
import orc  # noqa: E402  (the checker)
import rt_hip  # noqa: E402


# FUZZ_LARGE=1: images of 1,024 tiles and more, so launches take the host's
# heavy-first tile order with single, merged and tail tile groups
SIZES = [(1, 1), (7, 5), (64, 48), (96, 64), (160, 90)] if os.environ.get("FUZZ_LARGE") != "1" else \
    [(256, 256), (320, 240), (400, 300), (96, 64)]


def scene(rng):
    n = rng.choice([1, 2, 5, 30, 200, 700, 1100, 1500])
    spread = rng.choice([0.5, 5.0, 20.0, 1000.0])
    mirror = rng.random() < 0.3
    frac = rng.random() < 0.4  # fractional shininess: dd_pow (rt_pow.h) instead of int_pow

    def shin():
        if frac and rng.random() < 0.8:
            return "%.4f" % rng.choice([0.5, 7.5, 33.3, 1500.25, rng.uniform(0.01, 2000.0)])
        return "%d" % rng.choice([0, 1, 5, 20, 100, 200])

    lines = []
    for _ in range(n):
        r = rng.choice([1e-3, 0.05, 0.3, 1.0, 4.0]) * rng.uniform(0.5, 1.5) * spread / 10
        refl = rng.choice([0.8, 0.9, 1.0]) if mirror else rng.choice([0.0, 0.0, 0.3, 0.7, 1.0])
        lines.append("sphere %.9g %.9g %.9g %.9g %.3f %.3f %.3f %.2f 0.5 %s" % (
            rng.uniform(-spread, spread), rng.uniform(-spread, spread), rng.uniform(-3 * spread, spread), r,
            rng.random(), rng.random(), rng.random(), refl, shin()))
    near = os.environ.get("FUZZ_NEAR_LIGHTS") == "1"
    for _ in range(rng.randint(0, 6)):
        pos = (rng.uniform(-2 * spread, 2 * spread), rng.uniform(-spread, 3 * spread), rng.uniform(-3 * spread, spread))
        if near and n > 0 and rng.random() < 0.5:
            # FUZZ_NEAR_LIGHTS=1: a light just outside a sphere, within or near a shadow ray's
            # EPSILON overshoot past it (scene.h:72-82)
            f = lines[rng.randrange(n)].split()
            c, rad = [float(v) for v in f[1:4]], abs(float(f[4]))
            u = [rng.gauss(0, 1) for _ in range(3)]
            norm = sum(v * v for v in u) ** 0.5 or 1.0
            gap = rng.choice([0.0002, 0.0008, 0.00099, 0.0012, 0.003]) * rng.uniform(0.9, 1.1)
            pos = tuple(c[k] + u[k] / norm * (rad + gap) for k in range(3))
        lines.append("light %.9g %.9g %.9g %.3f %.3f %.3f 1" % (*pos, rng.random(), rng.random(), rng.random()))
    lines.append("ambient %.3f %.3f %.3f" % (rng.random() * 0.3, rng.random() * 0.3, rng.random() * 0.3))
    cam = [rng.uniform(-spread, spread) * 0.3 for _ in range(3)]
    look = [rng.uniform(-spread, spread) * 0.5, rng.uniform(-spread, spread) * 0.5, -2 * spread]
    lines.append("camera %.6g %.6g %.6g %.6g %.6g %.6g %d" % (*cam, *look, rng.choice([20, 45, 60, 90, 140])))
    return "\n".join(lines) + "\n"


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 300.0
    rng = random.Random(int(sys.argv[2]) if len(sys.argv) > 2 else 20261016)
    # FUZZ_VARIANT=tuning: the tuning build, so its RT_HIP_* knobs apply
    r = rt_hip.Renderer(0, variant=os.environ.get("FUZZ_VARIANT") or None)
    t0, k, px, frames, moving = time.time(), 0, 0, 0, 0
    try:
        while time.time() - t0 < budget:
            text = scene(rng)
            W, H, D = rng.choice(SIZES) + (rng.choice([0, 1, 2, 4, 8]),)
            sc = rt_hip.Scene.parse(text)
            r.upload(sc)
            rgb, st = r.render(sc.camera(), W, H, D)
            ref, cnt, _ = orc.OracleScene(text=text).render(W, H, D, threads=16)
            ok = bytes(rgb) == ref and (st.rays_primary, st.rays_shadow, st.rays_reflect) == (
                cnt["primary"], cnt["shadow"], cnt["reflect"])
            if ok and k % 3 == 2:  # three frames in one launch
                F, stride = 3, W * H * 3
                buf = torch.full((F * stride,), 77, dtype=torch.uint8, device="cuda:0")
                torch.cuda.synchronize()
                r.render_frames_async([sc.camera()] * F, W, H, D, None, buf.data_ptr(), stride)
                r.stats()
                host = bytes(buf.cpu().numpy())
                ok = all(host[f * stride:(f + 1) * stride] == ref for f in range(F))
                frames += F
                if ok:  # three frames from three camera positions: a device camera grid per frame
                    cams = []
                    for f in range(F):
                        c = rt_hip.rt_camera.from_buffer_copy(sc.camera())
                        for a in range(3):
                            c.position[a] += rng.uniform(-1.0, 1.0) * rng.choice([1e-3, 0.1, 1.0])
                        cams.append(c)
                    buf.fill_(77)
                    torch.cuda.synchronize()
                    r.render_frames_async(cams, W, H, D, None, buf.data_ptr(), stride)
                    st3 = r.stats()
                    host = bytes(buf.cpu().numpy())
                    oref = orc.OracleScene(text=text)
                    tot = [0, 0, 0]
                    for f in range(F):
                        want, c3, _ = oref.render(W, H, D, threads=16, camera=cams[f])
                        ok = ok and host[f * stride:(f + 1) * stride] == want
                        tot = [tot[0] + c3["primary"], tot[1] + c3["shadow"], tot[2] + c3["reflect"]]
                    ok = ok and [st3.rays_primary, st3.rays_shadow, st3.rays_reflect] == tot
                    moving += F
            k += 1
            px += W * H
            if not ok:
                bad = sum(a != b for a, b in zip(bytes(rgb), ref))
                print("MISMATCH scene %d (%dx%d d%d, %d spheres): %d bytes differ" % (
                    k, W, H, D, sc.num_spheres, bad), flush=True)
                with open(os.path.join(REPO, "gpurun_out", "fuzz_mismatch.txt"), "w") as f:
                    f.write("%d %d %d\n%s" % (W, H, D, text))
                return 1
            if k % 25 == 0:
                print("%d scenes ok (%d pixels), %.0f s" % (k, px, time.time() - t0), flush=True)
    finally:
        r.close()
    print("fuzz: %d scenes, %d pixels (+ %d frames of 3-frame launches at one position, %d frames of 3-frame "
          "launches at three positions), all byte-identical to the oracle" % (k, px, frames, moving))
    return 0


if __name__ == "__main__":
    sys.exit(main())
