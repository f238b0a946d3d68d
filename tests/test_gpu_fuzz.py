"""GPU: the randomised parity campaign, fixed seeds and a bounded budget, in
the driver-run suite (round 5's review: a light-grid defect -- a sphere
within a shadow ray's EPSILON overshoot past a light, scene.h:72-82 -- lived
through three driver-green rounds and was found only by the builder's
scripts/gpu_fuzz.py).

Every scene (tests/fuzz_gen.py) is rendered on cuda:0 through the C-ABI and
compared with the oracle byte for byte and ray count for ray count; every
third one also as three frames of one launch and three frames from three
camera positions.  Cases: the general generator (1-1,500 spheres, mirror
clouds, fractional shininess), lights just outside spheres, images of 1,024+
tiles, the EPSILON-margin generator (contact pairs, cameras and lights within
2 EPSILON of surfaces, exact tangents behind camera and reflection origins,
scenes 1e3-1e6 from the origin) with the camera grid built for every launch,
and a slice on the bounds-checked build (variants/librt_hip_check.so, where
an out-of-range structure index fails the render with RT_ERR_CHECK).  Each
case renders a fixed number of scenes of a fixed seed (deterministic), stops
early only past its time cap (a slow box), and requires at least its floor.
A second test puts random scenes through the other layouts of the same
arithmetic: rt_render_tiles (shuffled random tilings; the hybrid driver's and
launch_gpu_kernel's tile semantics, per-pixel stacks) and the 4-sample
antialias mode, against the oracle.
The parity bar is the reference's own: find_intersection / in_shadow / shade
/ trace_ray (scene.h:41-121, main.cpp:16-58) as the oracle restates them."""
import os
import random
import time

import pytest

import fuzz_gen
from conftest import diff_summary

pytestmark = pytest.mark.gpu

# (id, generator, sizes, seed, scenes, floor, cap seconds, variant, env)
CASES = [  # ~2,300 scenes, at most 80 s of caps (35 s for ~1,050 scenes on the round-6 box)
    ("general", "scene", fuzz_gen.SIZES, 20261018, 400, 200, 20.0, None, {}),
    ("near_lights", "near", fuzz_gen.SIZES, 7101, 450, 220, 16.0, None, {}),
    ("margin_camgrid", "margin", fuzz_gen.ODD_SIZES, 4242, 800, 400, 18.0, None, {"RT_HIP_CAM_GRID": "2"}),
    ("large_tiles", "near", fuzz_gen.LARGE_SIZES, 9090, 150, 60, 8.0, None, {}),
    ("checked_margin", "margin", fuzz_gen.ODD_SIZES, 77, 350, 150, 10.0, "check", {}),
    ("checked_near", "near", fuzz_gen.SIZES, 78, 150, 70, 8.0, "check", {}),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_random_scenes_byte_identical(case, monkeypatch):
    import orc
    import rt_hip
    import torch

    name, gen, sizes, seed, count, floor, cap, variant, env = case
    for k, v in env.items():
        monkeypatch.setenv(k, v)  # read by rt_create (product knobs)
    rng = random.Random(seed)
    r = rt_hip.Renderer(0, variant=variant)
    t0 = time.time()
    done = px = frames = moving = 0
    try:
        for k in range(count):
            if time.time() - t0 > cap:
                break
            if gen == "margin":
                text = fuzz_gen.margin_scene(rng)
            else:
                text = fuzz_gen.scene(rng, near=(gen == "near"))
            W, H = rng.choice(sizes)
            D = rng.choice([0, 1, 2, 4, 8])
            try:
                p, f, m = fuzz_gen.check_scene(r, text, W, H, D, rng, k, threads=16, torch=torch, orc=orc,
                                               rt_hip=rt_hip)
            except fuzz_gen.Mismatch as e:
                pytest.fail("fuzz[%s] seed %d scene %d (%dx%d d%d): %s\n%s" % (name, seed, k, W, H, D, e, text))
            done += 1
            px, frames, moving = px + p, frames + f, moving + m
    finally:
        r.close()
    print("fuzz[%s]: %d scenes, %d pixels, %d one-position and %d three-position launch frames, "
          "byte-identical to the oracle, %.1f s" % (name, done, px, frames, moving, time.time() - t0))
    assert done >= floor, f"only {done} scenes within {cap} s (floor {floor})"


# The other layouts of the same arithmetic on random scenes: rt_render_tiles
# (the hybrid driver's tile lists and the link-compatible launch_gpu_kernel,
# kernel.cu:185-207: per-pixel stacks, no merged levels, RGB8 tile semantics)
# against the oracle's full frame, and the 4-sample antialias mode
# (main_gpu.cu:249-333, serial fp64 semantics) against orc_render_aa.
# (id, generator, seed, scenes, floor, cap seconds): ~2,000 scenes in ~15 s on the round-6 box
LAYOUT_CASES = [("tiles_general", "scene", 31, 600, 200, 10.0), ("tiles_margin", "margin", 32, 600, 200, 8.0),
                ("antialias_general", "scene", 33, 400, 150, 10.0), ("antialias_margin", "margin", 34, 400, 150, 6.0)]


@pytest.mark.parametrize("case", LAYOUT_CASES, ids=[c[0] for c in LAYOUT_CASES])
def test_random_scenes_tiles_and_antialias(case, gpu_renderer):
    import orc
    import rt_hip
    import torch

    name, gen, seed, count, floor, cap = case
    rng = random.Random(seed)
    t0 = time.time()
    done = px = 0
    try:
        for k in range(count):
            if time.time() - t0 > cap:
                break
            text = fuzz_gen.margin_scene(rng) if gen == "margin" else fuzz_gen.scene(rng)
            W, H = rng.choice(fuzz_gen.ODD_SIZES if gen == "margin" else fuzz_gen.SIZES)
            D = rng.choice([0, 1, 2, 4, 8])
            sc = rt_hip.Scene.parse(text)
            gpu_renderer.upload(sc)
            o = orc.OracleScene(text=text)
            if name.startswith("tiles"):
                tw, th = rng.randint(1, max(1, W)), rng.randint(1, max(1, H))
                tiles = [(x, y, tw, th) for y in range(0, H, th) for x in range(0, W, tw)]
                rng.shuffle(tiles)
                buf = torch.full((W * H * 3,), 77, dtype=torch.uint8, device="cuda:0")
                torch.cuda.synchronize()
                gpu_renderer.render_tiles(sc.camera(), W, H, D, tiles, rt_hip.RT_FB_RGB8, buf.data_ptr())
                st = gpu_renderer.stats()
                got = bytes(buf.cpu().numpy())
                want, cnt, _ = o.render(W, H, D, threads=16)
            else:
                gpu_renderer.set_antialias(4)
                try:
                    rgb, st = gpu_renderer.render(sc.camera(), W, H, D)
                finally:
                    gpu_renderer.set_antialias(1)
                got = bytes(rgb)
                want, cnt, _ = o.render_aa(W, H, D, samples=4, threads=16)
            if got != want or (st.rays_primary, st.rays_shadow, st.rays_reflect) != (
                    cnt["primary"], cnt["shadow"], cnt["reflect"]):
                pytest.fail("fuzz[%s] seed %d scene %d (%dx%d d%d): %s; rays %s vs %s\n%s" % (
                    name, seed, k, W, H, D, diff_summary(got, want),
                    (st.rays_primary, st.rays_shadow, st.rays_reflect), cnt, text))
            done += 1
            px += W * H
    finally:
        gpu_renderer.set_antialias(1)
    print("fuzz[%s]: %d scenes, %d pixels, byte-identical to the oracle, %.1f s" % (name, done, px, time.time() - t0))
    assert done >= floor, f"only {done} scenes within {cap} s (floor {floor})"
