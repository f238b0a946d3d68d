"""GPU parity of multi-frame launches (rt_render_frames_async): every frame of a
launch is byte-identical to the golden image / to the single-frame render of
its own camera, and the launch's ray counts are the sums over its frames."""
import numpy as np
import pytest

from conftest import diff_summary, golden_rgb, manifest, scene_path, knob_variant

pytestmark = pytest.mark.gpu


def _load(r, name):
    import rt_hip

    m = manifest()[name]
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    r.upload(sc)
    return sc, m


def _frames(r, cams, W, H, D, rows=None, pad=0):
    """Render len(cams) frames in one launch; returns [F, R, W, 3] numpy and stats."""
    import torch

    R = rows.count if rows is not None else H
    stride = R * W * 3 + pad
    buf = torch.full((len(cams) * stride,), 77, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()  # the fill (torch's stream) lands before the render
    r.render_frames_async(cams, W, H, D, rows, buf.data_ptr(), stride)
    st = r.stats()
    host = buf.cpu().numpy()
    frames = np.stack([host[f * stride:f * stride + R * W * 3].reshape(R, W, 3) for f in range(len(cams))])
    gaps = [host[f * stride + R * W * 3:(f + 1) * stride] for f in range(len(cams))]
    return frames, st, gaps


def _single(r, cam, W, H, D, rows=None):
    rgb, st = r.render(cam, W, H, D, rows=rows)
    return bytes(rgb), st


def _moved(cam, k):
    """The scene camera moved sideways and zoomed a little, k steps (still a valid basis)."""
    import rt_hip

    c = rt_hip.rt_camera()
    for f in ("position", "forward", "right", "up"):
        getattr(c, f)[:] = list(getattr(cam, f))
    c.position[0] += 0.37 * k
    c.position[1] -= 0.11 * k
    c.scale = cam.scale * (1.0 + 0.05 * k)
    return c


@pytest.mark.parametrize("name,F", [("complex_97x61_d4", 2), ("complex_97x61_d4", 32), ("medium_1280x720_d10", 3),
                                    ("synth200_1920x1080_d4", 8), ("synth10k_384x216_d6", 5)])
def test_frames_equal_golden(gpu_renderer, name, F):
    sc, m = _load(gpu_renderer, name)
    frames, st, gaps = _frames(gpu_renderer, [sc.camera()] * F, m["width"], m["height"], m["depth"], pad=13)
    want = golden_rgb(name)
    for f in range(F):
        assert frames[f].tobytes() == want, f"frame {f}: {diff_summary(frames[f].tobytes(), want)}"
        assert (gaps[f] == 77).all(), "bytes between frames were written"
    rays = m["rays"]
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (F * rays["primary"], F * rays["shadow"],
                                                                   F * rays["reflect"])


def test_bench_launch_shape_equals_golden(gpu_renderer):
    """The bench's exact timed launch shapes on the metric workload (synth200
    1920x1080 d4, static camera: the camera grid on, frames packed with no gap
    so every tile row is dword aligned): a 32-frame launch (warmup, scratch
    sized), then a 20-frame one (the driver's --steps 20) and another 32-frame
    one, each frame equal to the reference's image."""
    name = "synth200_1920x1080_d4"
    sc, m = _load(gpu_renderer, name)
    W, H, D = m["width"], m["height"], m["depth"]
    want = golden_rgb(name)
    rays = m["rays"]
    for F in (32, 20, 32):
        frames, st, _ = _frames(gpu_renderer, [sc.camera()] * F, W, H, D)
        assert gpu_renderer.info().cam_grid_last == 1, "the static-view launch did not use the camera grid"
        for f in range(F):
            assert frames[f].tobytes() == want, f"F={F} frame {f}: {diff_summary(frames[f].tobytes(), want)}"
        assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (F * rays["primary"], F * rays["shadow"],
                                                                       F * rays["reflect"])


@pytest.mark.parametrize("name", ["complex_97x61_d4", "synth200_1920x1080_d4"])
def test_frames_distinct_cameras(gpu_renderer, name):
    sc, m = _load(gpu_renderer, name)
    W, H, D = m["width"], m["height"], m["depth"]
    cams = [_moved(sc.camera(), k) for k in (0, 3, -2, 1, 5, -4)]
    frames, st, _ = _frames(gpu_renderer, cams, W, H, D)
    total = [0, 0, 0]
    for f, cam in enumerate(cams):
        want, s1 = _single(gpu_renderer, cam, W, H, D)
        assert frames[f].tobytes() == want, f"frame {f}: {diff_summary(frames[f].tobytes(), want)}"
        total = [total[0] + s1.rays_primary, total[1] + s1.rays_shadow, total[2] + s1.rays_reflect]
    assert [st.rays_primary, st.rays_shadow, st.rays_reflect] == total
    assert frames[0].tobytes() == golden_rgb(name)  # k = 0 is the scene camera
    assert frames[1].tobytes() != frames[0].tobytes()


@pytest.mark.parametrize("G,band,F", [(3, 8, 4), (8, 8, 7), (5, 1, 2)])
def test_frames_row_shards(gpu_renderer, G, band, F):
    import rt_hip

    name = "complex_97x61_d4"
    sc, m = _load(gpu_renderer, name)
    W, H, D = m["width"], m["height"], m["depth"]
    cams = [_moved(sc.camera(), k) for k in range(F)]
    for r in range(G):
        rows = rt_hip.rows_for_shard(H, band, r, G)
        frames, _, _ = _frames(gpu_renderer, cams, W, H, D, rows)
        for f in range(F):
            want, _ = _single(gpu_renderer, cams[f], W, H, D, rows)
            assert frames[f].tobytes() == want, (r, f)


@pytest.mark.parametrize("depth", [0, 1, 2, 7])
def test_frames_depth_edges(gpu_renderer, depth):
    sc, m = _load(gpu_renderer, "complex_97x61_d4")
    cams = [_moved(sc.camera(), k) for k in (0, 2, 4)]
    frames, _, _ = _frames(gpu_renderer, cams, m["width"], m["height"], depth)
    for f, cam in enumerate(cams):
        want, _ = _single(gpu_renderer, cam, m["width"], m["height"], depth)
        assert frames[f].tobytes() == want, f


def test_frames_antialias(gpu_renderer):
    sc, m = _load(gpu_renderer, "complex_97x61_d4")
    cams = [_moved(sc.camera(), k) for k in (0, 1)]
    gpu_renderer.set_antialias(4)
    try:
        frames, _, _ = _frames(gpu_renderer, cams, m["width"], m["height"], m["depth"])
        for f, cam in enumerate(cams):
            want, _ = _single(gpu_renderer, cam, m["width"], m["height"], m["depth"])
            assert frames[f].tobytes() == want, f
    finally:
        gpu_renderer.set_antialias(1)


@pytest.mark.parametrize("env", [{"RT_HIP_LDS_SCENE": "1"}, {"RT_HIP_SCHED": "0"}, {"RT_HIP_STACK": "1"},
                                 {"RT_HIP_STACK": "4"}, {"RT_HIP_TAIL": "0"}],
                         ids=["lds-scene", "scanline", "global-stack", "merge", "no-single-tail"])
def test_frames_knobs(monkeypatch, env):
    import rt_hip

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    r = rt_hip.Renderer(0, variant=knob_variant())
    try:
        sc, m = _load(r, "synth200_1920x1080_d4")
        frames, _, _ = _frames(r, [sc.camera()] * 3, m["width"], m["height"], m["depth"])
        for f in range(3):
            assert frames[f].tobytes() == golden_rgb("synth200_1920x1080_d4"), f
    finally:
        r.close()


def test_frames_argument_errors(gpu_renderer):
    import torch
    import rt_hip

    sc, m = _load(gpu_renderer, "complex_97x61_d4")
    W, H, D = m["width"], m["height"], m["depth"]
    over = rt_hip.MAX_FRAMES + 1
    buf = torch.empty((over * H * W * 3,), dtype=torch.uint8, device="cuda:0")
    cam = sc.camera()
    for cams, stride in (([], H * W * 3), ([cam] * over, H * W * 3), ([cam] * 2, H * W * 3 - 1)):
        with pytest.raises(rt_hip.RtError):
            gpu_renderer.render_frames_async(cams, W, H, D, None, buf.data_ptr(), stride)
    # one frame ignores the stride, like rt_render_async
    gpu_renderer.render_frames_async([cam], W, H, D, None, buf.data_ptr(), 0)
    gpu_renderer.stats()
    assert buf[:H * W * 3].cpu().numpy().tobytes() == golden_rgb("complex_97x61_d4")


def test_camera_grid_rotated_views_one_position(gpu_renderer):
    """Eight views from one camera position in one launch (the camera grid is
    built for it: >= 8 frames at one position) -- looking at, beside, above and
    away from the scene -- each byte-identical to the oracle's render of that
    camera line (scene_loader.h camera grammar) with identical ray counts."""
    import orc
    import rt_hip

    base = open(scene_path("complex")).read()
    lines = [ln for ln in base.splitlines() if not ln.strip().startswith("camera")]
    targets = ["0 0 -20", "6 1 -20", "-8 3 -18", "0 9 -20", "0 -6 -15", "20 2 5", "0 3 40", "-3 -1 -60"]
    texts = ["\n".join(lines) + "\ncamera 0 3 12 %s 65\n" % t for t in targets]
    scenes = [rt_hip.Scene.parse(t) for t in texts]
    W, H, D = 64, 48, 4
    gpu_renderer.upload(scenes[0])
    frames, st, _ = _frames(gpu_renderer, [s.camera() for s in scenes], W, H, D)
    total = {"primary": 0, "shadow": 0, "reflect": 0}
    for f, t in enumerate(texts):
        ref, counts, _ = orc.OracleScene(text=t).render(W, H, D, threads=4)
        assert frames[f].tobytes() == ref, (targets[f], diff_summary(frames[f].tobytes(), ref))
        for k in total:
            total[k] += counts[k]
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (total["primary"], total["shadow"], total["reflect"])


def test_camera_grid_one_frame_policy(gpu_renderer):
    """One-frame launches (the drop-in's still frame): a position the previous
    launch did not use sweeps (no grid build for one frame), the same
    position's next launch builds and uses the device grid; both equal the
    reference's image, and a new position sweeps again."""
    name = "synth200_1920x1080_d4"
    sc, m = _load(gpu_renderer, name)
    W, H, D = m["width"], m["height"], m["depth"]
    want = golden_rgb(name)
    used = []
    for k in (1, 0, 0, 0, 2):
        rgb, _ = _single(gpu_renderer, _moved(sc.camera(), k), W, H, D)
        used.append(gpu_renderer.info().cam_grid_last)
        if k == 0:
            assert rgb == want, diff_summary(rgb, want)
    assert used == [0, 0, 1, 1, 0]


@pytest.mark.parametrize("F", [2, 17, 32])
def test_camera_grid_per_frame_device_grids(gpu_renderer, F):
    """A moving camera: one device-built camera grid per frame of the launch
    (every position distinct), each frame equal to its own one-frame render
    (the sweep: a new position per launch) with identical ray counts."""
    name = "complex_97x61_d4"
    sc, m = _load(gpu_renderer, name)
    W, H, D = m["width"], m["height"], m["depth"]
    cams = [_moved(sc.camera(), 0.25 * k - 3) for k in range(F)]
    frames, st, _ = _frames(gpu_renderer, cams, W, H, D)
    assert gpu_renderer.info().cam_grid_last == 1
    total = [0, 0, 0]
    for f, cam in enumerate(cams):
        want, s1 = _single(gpu_renderer, cam, W, H, D)
        assert frames[f].tobytes() == want, f"frame {f}: {diff_summary(frames[f].tobytes(), want)}"
        total = [total[0] + s1.rays_primary, total[1] + s1.rays_shadow, total[2] + s1.rays_reflect]
    assert [st.rays_primary, st.rays_shadow, st.rays_reflect] == total


@pytest.mark.parametrize("step", [1e-3, 0.21])
def test_camera_grid_moving_bench_shape_vs_oracle(gpu_renderer, step):
    """The bench's moving_camera shape pinned to the oracle: synth200 1920x1080
    d4 as ONE 32-frame launch of 32 distinct camera positions (the scene's
    basis, the position moved `step` further along x per frame, as bench.py's
    moved(); step 1e-3 is bench.py's own sequence), so 32 camera grids of N =
    128 are built on the device in the launch (camera.h:17-25 rays from each
    position, scene.h:41-61 closest hits).  Every 16th row of frames 0, 7, 19
    and 31 equals the oracle's render at that camera, and the launch's ray
    counts equal the oracle's full-frame counts summed over the 32 frames."""
    import orc
    import rt_hip

    name = "synth200_1920x1080_d4"
    sc, m = _load(gpu_renderer, name)
    W, H, D = m["width"], m["height"], m["depth"]
    F = rt_hip.MAX_FRAMES
    base = sc.camera()
    cams = []
    for f in range(F):
        c = rt_hip.rt_camera.from_buffer_copy(base)
        c.position[0] = base.position[0] + step * (f + 1)
        cams.append(c)
    frames, st, _ = _frames(gpu_renderer, cams, W, H, D)
    info = gpu_renderer.info()
    assert info.cam_grid_last == 1 and info.cam_grid_n == 128, (info.cam_grid_last, info.cam_grid_n)
    ref = orc.OracleScene(scene_path("synth200"))
    first, stride = 0, 16
    count = (H - first + stride - 1) // stride
    for f in (0, 7, 19, 31):
        rgb, _, _ = ref.render(W, H, D, band=1, first=first, stride=stride, count=count, threads=16, camera=cams[f])
        want = np.frombuffer(rgb, np.uint8).reshape(count, W, 3)
        for i in range(count):
            y = first + i * stride
            assert frames[f][y].tobytes() == want[i].tobytes(), \
                f"frame {f} row {y}: {diff_summary(frames[f][y].tobytes(), want[i].tobytes())}"
    total = [0, 0, 0]
    for f in range(F):
        _, cnt, _ = ref.render(W, H, D, threads=16, camera=cams[f])
        total = [total[0] + cnt["primary"], total[1] + cnt["shadow"], total[2] + cnt["reflect"]]
    assert [st.rays_primary, st.rays_shadow, st.rays_reflect] == total


@pytest.mark.parametrize("env", [{"RT_HIP_CAM_GRID_BUDGET": "0"}, {"RT_HIP_CAM_GRID_MAXP": "3"}],
                         ids=["no_budget", "pairs_dropped"])
def test_camera_grid_fallbacks(monkeypatch, env):
    """The camera grid is only a speed-up: with no memory budget for it the
    launch sweeps (no grid), and a grid whose (disk, block) pair list is cut
    short on the device is marked overflowed cell by cell (its rays sweep) --
    for a static view and a moving camera both, every frame equals the
    reference's image / its own one-frame render."""
    import rt_hip

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    r = rt_hip.Renderer(0, variant="tuning")
    try:
        name = "complex_97x61_d4"
        sc, m = _load(r, name)
        W, H, D = m["width"], m["height"], m["depth"]
        frames, _, _ = _frames(r, [sc.camera()] * 4, W, H, D)
        assert r.info().cam_grid_last == (0 if "RT_HIP_CAM_GRID_BUDGET" in env else 1)
        for f in range(4):
            assert frames[f].tobytes() == golden_rgb(name), f
        cams = [_moved(sc.camera(), 0.25 * k - 1) for k in range(5)]
        frames, _, _ = _frames(r, cams, W, H, D)
        for f, cam in enumerate(cams):
            want, _ = _single(r, cam, W, H, D)
            assert frames[f].tobytes() == want, f"frame {f}: {diff_summary(frames[f].tobytes(), want)}"
    finally:
        r.close()


@pytest.mark.parametrize("name", ["synth200_1920x1080_d4", "complex_1920x1080_d4", "complex_1280x720_d10",
                                  "mirrorfrac_320x240_d6", "complexfrac_960x540_d4", "medium_1920x1080_d2",
                                  "simple_800x600_d10", "synth10k_384x216_d6", "simple_2x2_d10"])
def test_wide_light_loop(monkeypatch, name):
    """The default kernels spread the light loop of sparse waves over their
    lanes (shade_hit kWide: a lane per (hit, light) for the shadow query and
    the Phong terms, each hit lane adding its lights' terms in file order,
    scene.h:94-120).  Against the reference's image and against the
    lane-per-ray loop (RT_HIP_WIDE=0, tuning build) from moved cameras, one
    frame and three per launch, ray counts included."""
    import rt_hip

    m = manifest()[name]
    W, H, D = m["width"], m["height"], m["depth"]
    r = rt_hip.Renderer(0)
    monkeypatch.setenv("RT_HIP_WIDE", "0")
    narrow = rt_hip.Renderer(0, variant="tuning")
    try:
        sc, _ = _load(r, name)
        narrow.upload(sc)
        rgb, st = _single(r, sc.camera(), W, H, D)
        assert rgb == golden_rgb(name), diff_summary(rgb, golden_rgb(name))
        for k in (1, -2):
            cam = _moved(sc.camera(), 0.3 * k)
            rgb, st = _single(r, cam, W, H, D)
            want, st0 = _single(narrow, cam, W, H, D)
            assert rgb == want, diff_summary(rgb, want)
            assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (st0.rays_primary, st0.rays_shadow,
                                                                          st0.rays_reflect)
        cams = [_moved(sc.camera(), 0.2 * k) for k in range(3)]
        frames, _, _ = _frames(r, cams, W, H, D)
        want, _, _ = _frames(narrow, cams, W, H, D)
        for f in range(len(cams)):
            assert frames[f].tobytes() == want[f].tobytes(), f"frame {f}"
    finally:
        r.close()
        narrow.close()


@pytest.mark.parametrize("seed", [3, 4])
def test_wide_mirror_cloud_vs_oracle(seed):
    """A camera inside a cloud of mirrors (most waves' deeper levels sparse,
    many rays deferred): the default (wide light loop) kernels against the
    oracle."""
    import orc
    import rt_hip
    from test_gpu_parity import _mirror_cloud

    text = _mirror_cloud(seed, 180, frac=seed == 4)
    sc = rt_hip.Scene.parse(text)
    r = rt_hip.Renderer(0)
    try:
        r.upload(sc)
        W, H, D = 160, 120, 7
        rgb, st = _single(r, sc.camera(), W, H, D)
        want, counts, _ = orc.OracleScene(text=text).render(W, H, D, threads=16)
        assert rgb == want, diff_summary(rgb, want)
        assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (counts["primary"], counts["shadow"],
                                                                      counts["reflect"])
    finally:
        r.close()
