"""Behind grid (rt_bvh.h build_ugrid, rt_device.h behind_cells).

With the grid, the ordered BVH walks of closest hits skip boxes wholly
behind the ray origin, and the part of the line behind the origin -- where
the reference's test (sphere.h:26-59) can only report the negative tangent
root of its disc == 0 branch (sphere.h:43-47) -- is checked by walking the
grid cells along it.

CPU: tests/native/ug_check.cpp runs the device's behind_cells on the host
for random scenes and lines, including lines built tangent to a sphere
behind their origin; every sphere the backward half-line is tangent to
(within 1e-7 of the diameter, and every exact disc == 0 case of the
reference's own arithmetic) must reach the exact test.

GPU: scenes where a camera ray or a reflection ray is EXACTLY tangent to a
sphere behind its origin (axis-aligned rays, so disc == 0 in the reference's
fp64 arithmetic and that sphere is the closest hit, at negative t), random
mirror clouds and the golden fixtures render byte-identical to the oracle
with the grid forced on (every closest hit walking the BVH), in one-frame
and multi-frame launches (the deferred walk kernel too), and with it off.
"""
import os
import subprocess

import pytest

from conftest import diff_summary, golden_rgb, manifest, scene_path, knob_variant

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "cs420-ray-tracer_amd", "csrc")


def test_behind_grid_covers_tangent_lines(tmp_path):
    """behind_cells and grid_closest_line, on the CPU (tests/native/ug_check.cpp)."""
    exe = tmp_path / "ug_check"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-I",
                    CSRC, "-I", os.path.join(REPO, "include"), "-o", str(exe),
                    os.path.join(REPO, "tests", "native", "ug_check.cpp"), os.path.join(CSRC, "rt_bvh.cpp")],
                   check=True)
    out = subprocess.run([str(exe), "24"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    first, second = out.stdout.strip().splitlines()[-2:]
    # "closest <lines> hits <count> wrong <count>": grid_closest_line == find_intersection
    c = first.split()
    assert c[0] == "closest" and int(c[1]) >= 90000 and int(c[3]) >= 40000 and c[-2:] == ["wrong", "0"]
    # "checked <lines> <near-tangent pairs> <exact disc0 pairs> scenes <used>/<built> cells/line <m> missed <k>"
    w = second.split()
    assert w[0] == "checked" and int(w[1]) >= 90000 and int(w[2]) >= 40000 and int(w[3]) >= 1000
    used, built = map(int, w[5].split("/"))
    assert used == built == 24
    assert w[-2] == "missed" and w[-1] == "0"


def _cloud(n, seed, mirrors=0.6):
    """A flat random cloud (synth10k-like, smaller) over a ground sphere."""
    import random

    rnd = random.Random(seed)
    lines = []
    for _ in range(n):
        x, y, z = rnd.uniform(-8, 8), rnd.uniform(-1, 4), rnd.uniform(-30, -6)
        r = rnd.uniform(0.15, 0.6)
        m = rnd.choice((0.0, 0.3, 0.6, 0.9)) if rnd.random() < mirrors else 0.0
        lines.append("sphere %.3f %.3f %.3f %.3f %.3f %.3f %.3f %.2f 0.5 %d\n" % (
            x, y, z, r, rnd.random(), rnd.random(), rnd.random(), m, rnd.choice((5, 10, 20, 50))))
    return "".join(lines)


TANGENT_SCENES = {
    # the centre pixel's camera ray is (0, 0, -1) exactly (W, H odd): its line is
    # tangent to the sphere at (0, 1, 5) behind the camera -- disc == 0, t = -5,
    # the closest hit
    "camera_ray": "sphere 0 1 5 1 0.9 0.2 0.2 0 0.5 10\nsphere 0 0 -10 3 0.2 0.9 0.2 0.5 0.5 20\n"
                  + _cloud(120, 7) + "sphere 0 -102 -20 100 0.3 0.3 0.3 0 1 5\n"
                  "light 0 12 -10 1 1 1 1\nlight 5 8 6 0.8 0.8 0.8 1\nambient 0.1 0.1 0.1\n"
                  "camera 0 0 0 0 0 -5 60\n",
    # the centre ray hits the mirror at (0, 0, -4) head on; its reflection leaves
    # (0, 0, -3.999) along +z, and that line is tangent to the sphere at
    # (0, 1, -12) behind the reflection's origin: disc == 0 exactly, t = -8.001
    "reflection_ray": "sphere 0 0 -5 1 0.9 0.9 0.9 0.9 0.5 50\nsphere 0 1 -12 1 0.1 0.3 0.9 0.2 0.5 10\n"
                      + _cloud(150, 11) + "sphere 0 -102 -20 100 0.3 0.3 0.3 0.3 1 5\n"
                      "light 0 12 -10 1 1 1 1\nlight -6 6 2 0.7 0.8 0.9 1\nambient 0.1 0.1 0.12\n"
                      "camera 0 0 0 0 0 -5 60\n",
}
W_T, H_T, D_T = 65, 49, 5  # odd: the centre pixel (32, 24) has u = v = 0.5 exactly


def test_tangent_scenes_need_the_negative_root():
    """The oracle's centre pixel changes when the tangent sphere is removed: the
    negative root is what these scenes test."""
    import orc

    for name, text in TANGENT_SCENES.items():
        drop = "sphere 0 1 5 1" if name == "camera_ray" else "sphere 0 1 -12 1"
        lines = [ln for ln in text.splitlines(True) if not ln.startswith(drop)]
        assert len(lines) == len(text.splitlines(True)) - 1
        ref, _, _ = orc.OracleScene(text=text).render(W_T, H_T, D_T, threads=4)
        ref2, _, _ = orc.OracleScene(text="".join(lines)).render(W_T, H_T, D_T, threads=4)
        c = (24 * W_T + 32) * 3
        assert ref[c:c + 3] != ref2[c:c + 3], name


_FORCED = {"RT_HIP_BEHIND_GRID": "1", "RT_HIP_BVH_ALWAYS": "1", "RT_HIP_SPHERE_GRID": "0", "RT_HIP_CAM_GRID": "0"}


@pytest.fixture(params=["on", "off", "on-defer1", "closest"])  # on*: BVH walk ahead + behind_cells
def behind_renderer(request, monkeypatch):
    import rt_hip

    env = dict(_FORCED)
    env["RT_HIP_GRID_CLOSEST"] = "0"
    if request.param == "off":
        env["RT_HIP_BEHIND_GRID"] = "0"
    if request.param == "on-defer1":
        env["RT_HIP_DEFER_LEVEL"] = "1"  # level >= 1 rays of multi-frame launches in the deferred walk kernel
    if request.param.startswith("closest"):
        env["RT_HIP_GRID_CLOSEST"] = "1"  # closest hits along the whole line through the grid, no BVH walk
        env["RT_HIP_DEFER_LEVEL"] = "1"
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    r = rt_hip.Renderer(0, variant=knob_variant())
    r.mode = request.param
    yield r
    r.close()


def _frames(r, cam, W, H, D, F):
    import numpy as np
    import torch

    stride = H * W * 3
    buf = torch.full((F * stride,), 77, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    r.render_frames_async([cam] * F, W, H, D, None, buf.data_ptr(), stride)
    r.stats()
    host = buf.cpu().numpy()
    return [bytes(host[f * stride:(f + 1) * stride]) for f in range(F)]


def _check(r, text, W, H, D, F=8):
    import orc
    import rt_hip

    sc = rt_hip.Scene.parse(text)
    r.upload(sc)
    ref, counts, _ = orc.OracleScene(text=text).render(W, H, D, threads=4)
    rgb, st = r.render(sc.camera(), W, H, D)
    info = r.info()
    assert bool(info.behind_grid_last) == (r.mode != "off")
    assert bytes(rgb) == ref, ("one frame", diff_summary(bytes(rgb), ref))
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (counts["primary"], counts["shadow"],
                                                                   counts["reflect"])
    for f, img in enumerate(_frames(r, sc.camera(), W, H, D, F)):
        assert img == ref, ("frame", f, diff_summary(img, ref))


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(TANGENT_SCENES))
def test_tangent_behind_vs_oracle(behind_renderer, name):
    _check(behind_renderer, TANGENT_SCENES[name], W_T, H_T, D_T)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_mirror_clouds_vs_oracle(behind_renderer, seed):
    text = (_cloud(400, 100 + seed, mirrors=0.9) + "sphere 0 -102 -20 100 0.3 0.3 0.3 0.5 1 5\n"
            "light 0 12 -10 1 1 1 1\nlight 10 10 -15 1 0.9 0.8 1\nlight -5 8 -20 0.9 1 1 1\n"
            "ambient 0.1 0.1 0.12\ncamera 0 3 12 0 0 -20 65\n")
    _check(behind_renderer, text, 96, 64, 6, F=4)


@pytest.mark.gpu
def test_goldens_with_behind_grid(monkeypatch):
    """Every golden fixture with the behind grid forced on (all closest hits walk)."""
    import rt_hip

    for k, v in _FORCED.items():
        monkeypatch.setenv(k, v)
    r = rt_hip.Renderer(0, variant=knob_variant())
    try:
        for name, m in sorted(manifest().items()):
            if m["width"] * m["height"] > 1280 * 720:
                continue
            sc = rt_hip.Scene.load(scene_path(m["scene"]))
            r.upload(sc)
            rgb, _ = r.render(sc.camera(), m["width"], m["height"], m["depth"])
            want = golden_rgb(name)
            assert bytes(rgb) == want, (name, diff_summary(bytes(rgb), want))
            info = r.info()
            assert info.behind_grid == (1 if sc.num_spheres > 0 else 0), name
            assert bool(info.behind_grid_last) == bool(info.behind_grid), name
    finally:
        r.close()


@pytest.mark.gpu
def test_default_uses_behind_grid_on_large_scenes(gpu_renderer):
    """synth10k (above kBvhAlwaysAbove spheres) gets the grid by default; its
    golden stays byte-identical (also covered by the golden tests)."""
    import rt_hip

    m = manifest()["synth10k_384x216_d6"]
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    gpu_renderer.upload(sc)
    rgb, _ = gpu_renderer.render(sc.camera(), m["width"], m["height"], m["depth"])
    info = gpu_renderer.info()
    assert info.behind_grid == 1 and info.behind_grid_last == 1 and info.behind_grid_entries > 0
    want = golden_rgb("synth10k_384x216_d6")
    assert bytes(rgb) == want, diff_summary(bytes(rgb), want)


@pytest.mark.gpu
@pytest.mark.parametrize("F", [2, 3, 7])
@pytest.mark.parametrize("W,H", [(40, 24), (97, 61)])
def test_xcd_frame_mapping_vs_oracle(monkeypatch, F, W, H):
    """Multi-frame launches with every frame of a tile group on one XCD
    (RT_HIP_XCD_FRAMES=1; the grid padded to a multiple of 8 groups): group
    counts that are not multiples of 8, odd frame counts, distinct cameras per
    frame -- every frame equals the oracle's render of its own camera."""
    import orc
    import rt_hip
    import torch

    monkeypatch.setenv("RT_HIP_XCD_FRAMES", "1")
    text = TANGENT_SCENES["reflection_ray"]
    sc = rt_hip.Scene.parse(text)
    r = rt_hip.Renderer(0, variant=knob_variant())
    try:
        r.upload(sc)
        base = sc.camera()
        cams = []
        for k in range(F):
            c = rt_hip.rt_camera.from_buffer_copy(base)
            c.position[0] = base.position[0] + 0.05 * k
            cams.append(c)
        stride = H * W * 3
        buf = torch.full((F * stride,), 77, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        r.render_frames_async(cams, W, H, 5, None, buf.data_ptr(), stride)
        r.stats()
        host = buf.cpu().numpy()
        for k in range(F):
            one, _ = r.render(cams[k], W, H, 5)
            got = bytes(host[k * stride:(k + 1) * stride])
            assert got == bytes(one), ("frame", k, diff_summary(got, bytes(one)))
            if k == 0:
                ref, _, _ = orc.OracleScene(text=text).render(W, H, 5, threads=4)
                assert got == ref, diff_summary(got, ref)
    finally:
        r.close()
