"""Shadow direction grids (rt_lightgrid.h).

CPU: the grid builder is conservative -- for random scenes (scales 0.1..1000,
far from the origin, tiny and huge spheres, grid sizes 1..64) every sphere the
reference's fp64 shadow test (sphere.h:26-59, scene.h:65-86) reports as an
occluder is on the list the device looks up (tests/native/lg_check.cpp).

GPU: scenes built to stress the grid (lights inside / on / next to spheres,
tiny occluders, a sphere tangent to axis-aligned shadow lines, far from the
origin) render byte-identical to the oracle with the grid at several
resolutions and with it disabled.
"""
import os
import subprocess

import pytest

from conftest import diff_summary, knob_variant

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "cs420-ray-tracer_amd", "csrc")


def test_grid_lists_are_conservative(tmp_path):
    exe = tmp_path / "lg_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", CSRC, "-o", str(exe),
                    os.path.join(REPO, "tests", "native", "lg_check.cpp"), os.path.join(CSRC, "rt_lightgrid.cpp")],
                   check=True)
    out = subprocess.run([str(exe), "40"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    far, words = [ln.split() for ln in out.stdout.strip().splitlines()[-2:]]
    assert words[0] == "checked" and int(words[1]) > 100000 and int(words[2]) > 100000
    assert words[-1] == "0"
    # small scenes 1e6 .. 1e10 from the origin (kLgOvershoot's absolute slack is
    # below their rounding; the relative margins must cover it)
    assert far[0] == "far" and int(far[1]) > 10000 and int(far[2]) > 30000, out.stdout


GRID_SCENES = {
    # the light sits exactly on a sphere's surface and inside another one
    "light_on_surface": "sphere 0 0 -5 1 0.8 0.2 0.2 0.3 1 10\nsphere 0 5 -5 2 0.2 0.8 0.2 0 1 10\n"
                        "sphere 0 -101 -5 100 0.5 0.5 0.5 0 1 5\nlight 0 1 -5 1 1 1 1\nlight 0 5 -5 0.5 0.5 0.5 1\n"
                        "camera 0 2 5 0 0 -5 60\n",
    # tiny occluders right next to the light, a huge sphere around everything
    "tiny_near_light": "".join("sphere %g %g %g 0.001 1 1 1 0 1 10\n" % (0.01 * i, 3 + 0.003 * i, -4 + 0.002 * i)
                               for i in range(-20, 20))
                       + "sphere 0 -101 -5 100 0.5 0.5 0.5 0.5 1 5\nsphere 0 0 -5 1 0.9 0.9 0.9 0.9 1 50\n"
                         "light 0 3.004 -4 1 1 1 1\ncamera 0 1 3 0 0 -5 70\n",
    # spheres just beyond lights (their surfaces 0.0002-0.0009 past them): a shadow ray starts EPSILON
    # past its point and runs EPSILON past the light (scene.h:72-82), into these spheres from any
    # direction -- the floor under the lights is in shadow (the light grids' global lists, kLgOvershoot);
    # one sphere 0.0015 away (beyond the overshoot: lit), and the fuzz scene's geometry (light 3 of
    # seed 7101 scene 4787: 0.00093 outside a sphere of radius 0.239)
    "sphere_beyond_light": "sphere 0 0.5005 -5 0.5 0.9 0.9 0.9 0 1 10\nlight 0 0 -5 1 1 1 1\n"
                           "sphere 2 0.3002 -5 0.3 0.2 0.9 0.2 0.5 1 20\nlight 2 0 -5 0.8 0.8 0.8 1\n"
                           "sphere -2 0.3015 -5 0.3 0.9 0.2 0.2 0 1 20\nlight -2 0 -5 0.7 0.7 0.7 1\n"
                           "sphere -0.23628557 0.493439321 -0.673393603 0.239067465 0.5 0.5 0.9 0 1 10\n"
                           "light -0.129703 0.285743 -0.729077 0.9 0.9 0.9 1\n"
                           "sphere 0 -101 -5 100 0.6 0.6 0.6 0.2 1 5\nambient 0.1 0.1 0.1\n"
                           "camera 0 1.5 3 0 -1 -5 75\n",
    # axis-aligned geometry: shadow lines along x = 0 graze spheres of radius 1 at x = +-1
    "axis_tangent": "sphere 1 2 -5 1 1 0 0 0 1 10\nsphere -1 4 -5 1 0 1 0 0.5 1 10\nsphere 0 -100 -5 100 1 1 1 0 1 1\n"
                    "sphere 1 -1 -5 1 0 0 1 0.2 1 10\nlight 0 10 -5 1 1 1 1\nlight 0 10 5 1 1 1 1\n"
                    "camera 0 1 5 0 1 -5 60\n",
    # lights scattered inside a dense mirror cluster
    "lights_in_cluster": "".join("sphere %g %g %g %g 0.7 0.7 0.7 %g 1 20\n" % (
        (i * 7919 % 100) / 10 - 5, (i * 104729 % 100) / 10 - 5, (i * 1299709 % 100) / 10 - 25, 0.3 + (i % 5) * 0.2,
        (i % 4) * 0.3) for i in range(150))
                         + "".join("light %g %g %g 0.3 0.3 0.3 1\n" % ((l * 37 % 10) - 5, (l * 53 % 10) - 5,
                                                                       -25 + (l * 71 % 10)) for l in range(6))
                         + "ambient 0.05 0.05 0.05\ncamera 0 0 0 0 0 -25 60\n",
    # the same cluster translated far from the origin
    "far_cluster": "".join("sphere %g %g %g %g 0.7 0.7 0.7 %g 1 20\n" % (
        1e6 + (i * 7919 % 100) / 10 - 5, 1e6 + (i * 104729 % 100) / 10 - 5, -1e6 + (i * 1299709 % 100) / 10 - 25,
        0.3 + (i % 5) * 0.2, (i % 4) * 0.3) for i in range(120))
                   + "light 1000000 1000008 -1000020 1 1 1 1\nlight 999995 1000000 -1000025 0.5 0.5 0.5 1\n"
                     "camera 1000000 1000000 -1000000 1000000 1000000 -1000025 60\n",
}


@pytest.fixture(params=[("1", "64"), ("1", "1"), ("1", "2"), ("1", "7"), ("0", "64")],
                ids=["grid64", "grid1", "grid2", "grid7", "nogrid"])
def grid_renderer(request, monkeypatch):
    import rt_hip

    on, n = request.param
    monkeypatch.setenv("RT_HIP_SHADOW_GRID", on)
    monkeypatch.setenv("RT_HIP_SHADOW_GRID_N", n)
    r = rt_hip.Renderer(0, variant=knob_variant())
    yield r
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GRID_SCENES))
def test_grid_scenes_vs_oracle(grid_renderer, name):
    import orc
    import rt_hip

    text = GRID_SCENES[name]
    W, H, D = 96, 72, 5
    sc = rt_hip.Scene.parse(text)
    grid_renderer.upload(sc)
    ref, counts, _ = orc.OracleScene(text=text).render(W, H, D, threads=4)
    rgb, st = grid_renderer.render(sc.camera(), W, H, D)
    assert bytes(rgb) == ref, diff_summary(bytes(rgb), ref)
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (counts["primary"], counts["shadow"],
                                                                   counts["reflect"])


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"RT_HIP_STACK": "1"}, {"RT_HIP_LDS_SCENE": "1"}], ids=["global-stack", "lds-scene"])
def test_grid_in_other_layouts(monkeypatch, env):
    import orc
    import rt_hip

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    r = rt_hip.Renderer(0, variant=knob_variant())
    try:
        for name in ("lights_in_cluster", "axis_tangent"):
            text = GRID_SCENES[name]
            sc = rt_hip.Scene.parse(text)
            r.upload(sc)
            ref, _, _ = orc.OracleScene(text=text).render(80, 60, 6, threads=4)
            rgb, _ = r.render(sc.camera(), 80, 60, 6)
            assert bytes(rgb) == ref, (name, diff_summary(bytes(rgb), ref))
    finally:
        r.close()


def test_own_sphere_pretest_agrees_with_reference(tmp_path):
    """shadow_cells decides the shaded point's own sphere before its lists
    (rt_device.h): "in shadow" when the ray origin is inside it and
    dist^2 > 6 r^2, "skip" when both roots are provably negative.  Both must
    agree with the reference's test of that sphere (sphere.h:26-59 +
    scene.h:78-82) on 4M random shaded points, grazing hits and lights on, near
    and inside the sphere (tests/native/self_check.cpp)."""
    exe = tmp_path / "self_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(REPO, "tests", "native", "self_check.cpp")], check=True)
    out = subprocess.run([str(exe), "4000000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    w = out.stdout.split()
    assert w[0] == "checked" and int(w[1]) > 3000000 and int(w[3]) > 100000 and int(w[5]) > 100000
    assert w[-1] == "0", out.stdout


def test_sqrt_free_decisions_agree_with_reference(tmp_path):
    """intersect_num decides two cases of disc > 0 without the square root
    (rt_device.h): b > 0 with disc < b^2 (1 - 2^-50) is a miss (both roots
    negative), and c > 0, b < 0 with -b below a shadow query's bound is an
    occluder (0 <= n1 <= -b).  On 8M shadow pairs (spheres along the query's
    line: between the point and the light, beyond either, through the origin,
    grazing within |r| 10^-15, exactly tangent to axis-aligned lines) and 16M
    closest-hit pairs, the decisions equal the reference's test (sphere.h:26-59,
    scene.h:78-82) and every returned numerator gives its t exactly; and the
    bound that lets shadow_cells skip its per-ray line check (off_free) holds
    (tests/native/num_check.cpp)."""
    exe = tmp_path / "num_check"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-I",
                    os.path.join(REPO, "cs420-ray-tracer_amd", "csrc"), "-I", os.path.join(REPO, "include"), "-o",
                    str(exe), os.path.join(REPO, "tests", "native", "num_check.cpp")], check=True)
    out = subprocess.run([str(exe), "1000000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    sh, cl, off = out.stdout.strip().splitlines()[-3:]
    w = sh.split()
    assert w[0] == "shadow" and int(w[1]) > 7000000 and int(w[5]) > 500000 and int(w[7]) > 500000, sh
    assert w[-1] == "0", sh
    c = cl.split()
    assert c[0] == "closest" and int(c[3]) > 5000000 and c[-1] == "0", cl
    # shadow_cells' off_free: the computed line-to-light distance under 2^-41 (1.01 B + 0.01)
    f = off.split()
    assert f[0] == "off" and int(f[1]) > 100000 and float(f[3]) < 0.01 and f[-1] == "0", off


def test_camera_grid_lists_and_scan(tmp_path):
    """Camera grid (rt_lightgrid.h build_point_grid, rt_device.h cam_closest):
    every sphere the reference's test reports a hit for on a camera ray, with
    t of either sign, is on the looked-up cell's list (device binning and its
    +-2^-22 quotient errors) with tlo <= t, and the early-exit scan returns
    find_intersection's (t, index) -- random scenes at scales 0.1..1000, far
    from the origin, negative radii, cameras inside / on spheres, rays aimed at
    silhouettes ahead of and behind the camera (tests/native/cg_check.cpp)."""
    exe = tmp_path / "cg_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", CSRC, "-o", str(exe),
                    os.path.join(REPO, "tests", "native", "cg_check.cpp"), os.path.join(CSRC, "rt_lightgrid.cpp")],
                   check=True)
    out = subprocess.run([str(exe), "40"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    w = out.stdout.split()
    assert w[0] == "checked" and int(w[1]) > 100000 and int(w[2]) > 200000, out.stdout
    assert w[4] == "0" and w[6] == "0", out.stdout


def test_camera_grid_device_builder(tmp_path):
    """The device camera-grid builder's per-lane functions (csrc/rt_cgbuild.h,
    shared with rt_kernel.hip's cg_disk / cg_bin kernels) run lane by lane in
    the kernels' pass structure on the CPU, 1-3 grids per scene
    (tests/native/cg_device_check.cpp): every cell within its 48 slots lists
    exactly build_point_grid's entries in (tlo, index) order, every sphere the
    reference's test reports on a camera ray (either sign of t) is on the
    looked-up list with tlo <= t, and cam_closest's early-exit scan returns
    find_intersection's (t, index) -- the same random scenes, cameras and
    silhouette rays as the host-builder check."""
    exe = tmp_path / "cg_device_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", CSRC, "-o", str(exe),
                    os.path.join(REPO, "tests", "native", "cg_device_check.cpp"),
                    os.path.join(CSRC, "rt_lightgrid.cpp"), "-lpthread"], check=True)
    out = subprocess.run([str(exe), "60"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    w = out.stdout.split()
    assert w[0] == "checked" and int(w[1]) > 100000 and int(w[2]) > 200000 and int(w[4]) > 5000000, out.stdout
    assert w[8] == "0" and w[10] == "0" and w[12] == "0", out.stdout


def test_sphere_grid_device_builder_matches_host(tmp_path):
    """The device point-grid builder (rt_kernel.hip pg_disk / pg_bin / scan /
    sort / start kernels, per-lane functions shared through
    csrc/rt_cgbuild.h) run lane by lane in its pass structure on the CPU
    (tests/native/sg_device_check.cpp) gives, on 120 random scenes (scales
    0.1-1000, far from the origin, negative and tiny radii, a ground-sized
    sphere, dense clusters whose grids exceed the global-sphere cap), the same
    grid spheres, the same refusals and, for every cell of every grid, exactly
    build_sphere_grids' list (sphere, tlo bits) in the same order -- so the
    host builder's proofs (tests/native/sg_check.cpp) carry over; and for the
    light grids (1-6 lights per scene, one at a sphere's centre, some
    non-finite) exactly build_light_grid's start rows and, list by list, the
    same ids -- the device orders them nearest first (ids_sort_kernel), the
    host by id; a shadow query is an any-hit test, so the order is free
    (tests/native/lg_check.cpp's proofs carry over)."""
    exe = tmp_path / "sg_device_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", CSRC, "-o", str(exe),
                    os.path.join(REPO, "tests", "native", "sg_device_check.cpp"),
                    os.path.join(CSRC, "rt_lightgrid.cpp"), "-lpthread"], check=True)
    out = subprocess.run([str(exe), "120"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    w = out.stdout.split()
    assert w[0] == "scenes" and int(w[3]) > 3000 and int(w[5]) > 500 and int(w[9]) > 10000000, out.stdout
    assert w[11] == "0", out.stdout
    # the light grids (one side, a separate global list, nearest first) against build_light_grid
    assert w[12] == "lights" and int(w[13]) > 300 and int(w[15]) > 5000000 and w[17] == "0", out.stdout


CAM_SCENES = dict(GRID_SCENES)
CAM_SCENES.update({
    # the camera inside a mirror sphere that holds the other spheres
    "camera_inside": "sphere 0 0 -3 20 0.9 0.9 0.9 0.8 1 20\nsphere 0 0 -6 1 1 0 0 0.5 1 10\n"
                     "sphere 2 1 -4 0.5 0 1 0 0.9 1 50\nsphere -2 -1 3 1 0 0 1 0.3 1 5\n"
                     "light 0 5 -3 1 1 1 1\ncamera 0 0 0 0 0 -6 70\n",
    # the camera exactly on a sphere's surface, spheres behind it and a negative radius
    "camera_on_surface": "sphere 0 0 1 1 0.5 0.5 0.5 0.5 1 10\nsphere 0 0 -6 -1.5 1 0.5 0 0.4 1 20\n"
                         "sphere 3 0 4 1 0 1 1 0.6 1 10\nsphere 0 -101 -5 100 0.5 0.5 0.5 0.2 1 5\n"
                         "light 4 6 2 1 1 1 1\ncamera 0 0 0 0 0 -6 80\n",
})


@pytest.fixture(params=["512", "64", "7", "1"], ids=lambda n: "camgrid" + n)
def camgrid_renderer(request, monkeypatch):
    import rt_hip

    monkeypatch.setenv("RT_HIP_CAM_GRID", "2")
    monkeypatch.setenv("RT_HIP_CAM_GRID_N", request.param)
    r = rt_hip.Renderer(0, variant=knob_variant())
    yield r
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CAM_SCENES))
def test_camera_grid_scenes_vs_oracle(camgrid_renderer, name):
    import orc
    import rt_hip

    text = CAM_SCENES[name]
    W, H, D = 96, 72, 5
    sc = rt_hip.Scene.parse(text)
    camgrid_renderer.upload(sc)
    ref, counts, _ = orc.OracleScene(text=text).render(W, H, D, threads=4)
    rgb, st = camgrid_renderer.render(sc.camera(), W, H, D)
    assert bytes(rgb) == ref, diff_summary(bytes(rgb), ref)
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (counts["primary"], counts["shadow"],
                                                                   counts["reflect"])


@pytest.mark.gpu
def test_camera_grid_goldens(monkeypatch):
    """Every golden fixture through the camera grid (forced) is byte-identical."""
    import rt_hip
    from conftest import golden_rgb, manifest, scene_path

    monkeypatch.setenv("RT_HIP_CAM_GRID", "2")
    r = rt_hip.Renderer(0, variant=knob_variant())
    try:
        for name, m in sorted(manifest().items()):
            sc = rt_hip.Scene.load(scene_path(m["scene"]))
            r.upload(sc)
            rgb, st = r.render(sc.camera(), m["width"], m["height"], m["depth"])
            want = golden_rgb(name)
            assert bytes(rgb) == want, (name, diff_summary(bytes(rgb), want))
    finally:
        r.close()


def test_sphere_grid_lists_and_scan(tmp_path):
    """Sphere grids (rt_lightgrid.h build_sphere_grids, rt_device.h
    grid_closest): for reflection rays built as the renderer builds them
    (origin hit point + normal * 0.001, the reflected direction) and rays from
    those origins aimed at silhouettes ahead and behind, whose origin passes
    the device's ball check, every sphere the reference's test reports a hit
    for (t of either sign) is on the looked-up cell's list of the grid of the
    sphere the ray leaves with tlo <= t, and the early-exit scan returns
    find_intersection's (t, index) -- random scenes at scales 0.1..1000, far
    from the origin, negative and tiny radii, a ground sphere
    (tests/native/sg_check.cpp)."""
    exe = tmp_path / "sg_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", CSRC, "-o", str(exe),
                    os.path.join(REPO, "tests", "native", "sg_check.cpp"), os.path.join(CSRC, "rt_lightgrid.cpp"),
                    "-lpthread"], check=True)
    out = subprocess.run([str(exe), "40"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    w = out.stdout.split()
    assert w[0] == "checked" and int(w[1]) > 100000 and int(w[2]) > 200000, out.stdout
    # the origin check passes for every renderer-built ray; missed = wrong = 0
    assert int(w[4]) <= int(w[1]) // 1000 and w[6] == "0" and w[8] == "0", out.stdout


@pytest.fixture(params=["16", "4", "1", "off"], ids=lambda n: "spheregrid" + n)
def spheregrid_renderer(request, monkeypatch):
    import rt_hip

    if request.param == "off":
        monkeypatch.setenv("RT_HIP_SPHERE_GRID", "0")
    else:
        monkeypatch.setenv("RT_HIP_SPHERE_GRID", "1")
        monkeypatch.setenv("RT_HIP_SPHERE_GRID_N", request.param)
    r = rt_hip.Renderer(0, variant=knob_variant())
    yield r, request.param
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CAM_SCENES))
def test_sphere_grid_scenes_vs_oracle(spheregrid_renderer, name):
    """Reflection rays through the sphere grids (single and 8-frame launches,
    the latter with the deferred kernel) against the oracle."""
    import orc
    import rt_hip

    import torch

    r, mode = spheregrid_renderer
    text = CAM_SCENES[name]
    W, H, D = 96, 72, 6
    sc = rt_hip.Scene.parse(text)
    r.upload(sc)
    info = r.info().as_dict()
    assert (info["sphere_grids"] > 0) == (mode != "off"), info  # every scene here has mirrors
    ref, counts, _ = orc.OracleScene(text=text).render(W, H, D, threads=4)
    rgb, st = r.render(sc.camera(), W, H, D)
    assert bytes(rgb) == ref, diff_summary(bytes(rgb), ref)
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (counts["primary"], counts["shadow"],
                                                                   counts["reflect"])
    buf = torch.zeros((8, H, W, 3), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    r.render_frames_async([sc.camera()] * 8, W, H, D, None, buf.data_ptr(), H * W * 3)
    r.stats()  # waits for the launch
    for f in range(8):
        got = bytes(buf[f].cpu().numpy().tobytes())
        assert got == ref, (f, diff_summary(got, ref))


@pytest.mark.gpu
def test_sphere_grid_goldens(monkeypatch):
    """Every golden fixture with the sphere grids forced on, at two N, is
    byte-identical (the default turns them on up to 2,048 spheres)."""
    import rt_hip
    from conftest import golden_rgb, manifest, scene_path

    for n in ("16", "3"):
        monkeypatch.setenv("RT_HIP_SPHERE_GRID", "1")
        monkeypatch.setenv("RT_HIP_SPHERE_GRID_N", n)
        r = rt_hip.Renderer(0, variant=knob_variant())
        try:
            for name, m in sorted(manifest().items()):
                sc = rt_hip.Scene.load(scene_path(m["scene"]))
                r.upload(sc)
                # above 2,048 spheres even a forced build gives up (the entry cap)
                assert r.info().sphere_grids > 0 or sc.num_spheres > 2048, name
                rgb, st = r.render(sc.camera(), m["width"], m["height"], m["depth"])
                want = golden_rgb(name)
                assert bytes(rgb) == want, (name, n, diff_summary(bytes(rgb), want))
        finally:
            r.close()


@pytest.mark.gpu
def test_sphere_grids_built_lazily(monkeypatch):
    """Default policy: rt_upload_scene builds no sphere grids; a scene's first
    one-frame launch sweeps, its second launch (or a first multi-frame launch)
    builds them -- every render equal to the golden either way."""
    import rt_hip
    import torch
    from conftest import golden_rgb, manifest, scene_path

    monkeypatch.delenv("RT_HIP_SPHERE_GRID", raising=False)
    name = "complex_97x61_d4"
    m = manifest()[name]
    want = golden_rgb(name)
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    r = rt_hip.Renderer(0)
    try:
        W, H, D = m["width"], m["height"], m["depth"]
        r.upload(sc)
        assert r.info().sphere_grids == 0
        rgb, _ = r.render(sc.camera(), W, H, D)
        assert bytes(rgb) == want and r.info().sphere_grids == 0
        rgb, _ = r.render(sc.camera(), W, H, D)
        assert bytes(rgb) == want and r.info().sphere_grids > 0
        r.upload(sc)  # a new upload: pending again; a 3-frame launch builds them at once
        assert r.info().sphere_grids == 0
        buf = torch.zeros((3, H, W, 3), dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        r.render_frames_async([sc.camera()] * 3, W, H, D, None, buf.data_ptr(), H * W * 3)
        r.stats()
        assert r.info().sphere_grids > 0
        for f in range(3):
            assert buf[f].cpu().numpy().tobytes() == want, f
    finally:
        r.close()
