"""GPU: scenes far past the benchmark's sizes -- 60,000, 250,000 and 1,000,000
spheres (synth10k, BASELINE cfg 5, is the largest elsewhere in the suite) -- through
the product library, byte for byte and ray count for ray count against the
oracle's brute-force find_intersection / in_shadow / trace_ray
(scene.h:41-121, main.cpp:16-58), in a one-frame launch and in a
three-frame launch (merged levels, the deferred queue).  At these sizes the
upload builds the BVH and the uniform grid on the host and the light grids on
the device, past the sphere grids' limit (2,048 spheres); the images are
small so that the oracle's brute force over every sphere stays within
seconds."""
import random
import time

import pytest

from conftest import diff_summary

pytestmark = pytest.mark.gpu


def _cloud(n: int, seed: int) -> str:
    """A synth10k-like cloud (SURVEY 8(d)'s generator shape, denser and wider)
    over a ground sphere, complex.txt's lights and camera."""
    rnd = random.Random(seed)
    lines = []
    for _ in range(n - 1):
        lines.append("sphere %.3f %.3f %.3f %.3f %.3f %.3f %.3f %.2f 0.5 %d\n" % (
            rnd.uniform(-80, 80), rnd.uniform(-1.5, 20), rnd.uniform(-240, -15), rnd.uniform(0.1, 0.45),
            rnd.random(), rnd.random(), rnd.random(), rnd.choice((0.0, 0.0, 0.3, 0.6, 0.9)),
            rnd.choice((5, 10, 20, 50, 100))))
    lines.append("sphere 0 -102 -20 100 0.3 0.3 0.3 0 1 5\n")
    lines.append("light -10 10 -10 1 0.9 0.8 1\nlight 10 15 -20 0.8 0.9 1 1\nlight 0 20 -30 1 1 1 1\n"
                 "light -20 5 -5 0.6 0.6 0.8 1\nlight 20 8 -15 0.9 0.7 0.6 1\nambient 0.1 0.1 0.12\n"
                 "camera 0 3 12 0 0 -20 65\n")
    return "".join(lines)


# (id, spheres, W, H, depth)
CASES = [("cloud60k", 60000, 96, 64, 4), ("cloud250k", 250000, 48, 32, 4), ("cloud1m", 1000000, 32, 24, 3)]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_large_scene_byte_identical(case):
    import orc
    import rt_hip
    import torch

    name, n, W, H, D = case
    text = _cloud(n, seed=n)
    sc = rt_hip.Scene.parse(text)
    assert sc.num_spheres == n
    r = rt_hip.Renderer(0)
    try:
        t0 = time.time()
        r.upload(sc)
        t_up = time.time() - t0
        want, cnt, t_orc = orc.OracleScene(text=text).render(W, H, D, threads=16)
        rays = (cnt["primary"], cnt["shadow"], cnt["reflect"])
        # one frame
        rgb, st = r.render(sc.camera(), W, H, D)
        got = bytes(rgb)
        assert got == want, "%s one frame: %s" % (name, diff_summary(got, want))
        assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == rays
        # three frames of one view in one launch (merged levels, deferred queue)
        buf = torch.full((3 * W * H * 3,), 77, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        r.render_frames_async([sc.camera()] * 3, W, H, D, None, buf.data_ptr(), W * H * 3)
        st3 = r.stats()
        frames = bytes(buf.cpu().numpy())
        for f in range(3):
            part = frames[f * W * H * 3:(f + 1) * W * H * 3]
            assert part == want, "%s frame %d of 3: %s" % (name, f, diff_summary(part, want))
        assert (st3.rays_primary, st3.rays_shadow, st3.rays_reflect) == tuple(3 * x for x in rays)
    finally:
        r.close()
    print("%s: %d spheres, %dx%d d%d, %d rays, upload %.2f s, oracle %.1f s: byte-identical" % (
        name, n, W, H, D, sum(rays), t_up, t_orc))


def test_large_scene_wide_image_sampled_rows():
    """60,000 spheres at 1280x720 depth 4 (a launch of 14,400 tiles: the
    heavy-first tile order, merged waves, the launch tail, the deferred queue's
    shards) against the oracle on every 23rd row."""
    import orc
    import rt_hip

    W, H, D, stride = 1280, 720, 4, 23
    text = _cloud(60000, seed=7)
    sc = rt_hip.Scene.parse(text)
    r = rt_hip.Renderer(0)
    try:
        r.upload(sc)
        rgb, st = r.render(sc.camera(), W, H, D)
    finally:
        r.close()
    rows = list(range(3, H, stride))
    want, cnt, dt = orc.OracleScene(text=text).render(W, H, D, band=1, first=3, stride=stride, count=len(rows),
                                                      threads=16)
    got = b"".join(bytes(rgb[y * W * 3:(y + 1) * W * 3]) for y in rows)
    assert got == want, diff_summary(got, want)
    print("cloud60k 1280x720 d4: %d sampled rows byte-identical (oracle %.1f s), %d rays in the frame" % (
        len(rows), dt, st.rays_primary + st.rays_shadow + st.rays_reflect))
