"""GPU: the bounds-checked build (variants/librt_hip_check.so, -DRT_CHECK;
SURVEY 5's HIP bounds-checked debug build, the analogue of the reference's
memory-check pass, scripts/test.sh:175-194).  Every indirect device index
into a host-built structure -- light / camera / sphere grid CSR starts and
ids, uniform-grid cells and overflow lists, BVH nodes and leaf slots, the
tile order, deferred-queue, reflection-stack, LDS queue and pixel slots,
framebuffer offsets -- is range-checked; a violation makes rt_render_stats
return RT_ERR_CHECK with the site's name, which these renders would raise.
Each render must also equal the reference's image (or the oracle)."""
import os

import numpy as np
import pytest

from conftest import diff_summary, golden_rgb, manifest, scene_path

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def check_renderer():
    import rt_hip

    r = rt_hip.Renderer(0, variant="check")
    yield r
    r.close()


@pytest.mark.parametrize("name", ["complex_97x61_d4", "medium_1280x720_d10", "synth200_1920x1080_d4",
                                  "mirrorfrac_320x240_d6", "synth10k_384x216_d6"])
def test_checked_goldens(check_renderer, name):
    import rt_hip

    m = manifest()[name]
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    check_renderer.upload(sc)
    rgb, st = check_renderer.render(sc.camera(), m["width"], m["height"], m["depth"])  # raises on RT_ERR_CHECK
    want = golden_rgb(name)
    assert bytes(rgb) == want, diff_summary(bytes(rgb), want)


@pytest.mark.parametrize("name,F", [("synth200_1920x1080_d4", 8), ("synth10k_384x216_d6", 5)])
def test_checked_multi_frame_launch(check_renderer, name, F):
    """Multi-frame launches: camera grid, deferred kernel, frame-strided output."""
    import rt_hip
    import torch

    m = manifest()[name]
    W, H, D = m["width"], m["height"], m["depth"]
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    check_renderer.upload(sc)
    buf = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    check_renderer.render_frames_async([sc.camera()] * F, W, H, D, None, buf.data_ptr(), H * W * 3)
    check_renderer.stats()  # raises on RT_ERR_CHECK
    host = buf.cpu().numpy()
    want = golden_rgb(name)
    for f in range(F):
        assert host[f].tobytes() == want, f"frame {f}: {diff_summary(host[f].tobytes(), want)}"


@pytest.mark.parametrize("name,F", [("synth200_1920x1080_d4", 32), ("complex_97x61_d4", 5)])
def test_checked_moving_camera_launch(check_renderer, name, F):
    """A moving camera in the checked build: F camera positions in one launch,
    so the device builds a camera grid per frame (cg_disk / cg_bin / cg_sort,
    their pair, count and slot indices checked) and every frame's scan reads
    its own grid; each frame equals the oracle at its camera (every 24th row
    at 1080p)."""
    import orc
    import rt_hip
    import torch

    m = manifest()[name]
    W, H, D = m["width"], m["height"], m["depth"]
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    check_renderer.upload(sc)
    cams = []
    for f in range(F):
        c = rt_hip.rt_camera.from_buffer_copy(sc.camera())
        c.position[0] += 0.05 * (f + 1)
        c.position[2] -= 0.03 * f
        cams.append(c)
    buf = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    check_renderer.render_frames_async(cams, W, H, D, None, buf.data_ptr(), H * W * 3)
    check_renderer.stats()  # raises on RT_ERR_CHECK
    assert check_renderer.info().cam_grid_last == 1
    host = buf.cpu().numpy()
    ref = orc.OracleScene(scene_path(m["scene"]))
    step = 24 if H > 200 else 1
    count = (H + step - 1) // step
    for f in (0, F // 2, F - 1):
        rgb, _, _ = ref.render(W, H, D, stride=step, count=count, threads=16, camera=cams[f])
        want = np.frombuffer(rgb, np.uint8).reshape(count, W, 3)
        for i in range(count):
            assert host[f][i * step].tobytes() == want[i].tobytes(), f"frame {f} row {i * step}"


def test_checked_deferred_queue_overflow(monkeypatch):
    """A camera inside a cloud of mirrors (test_gpu_parity._mirror_cloud):
    level-2 rays overflow the deferred queue; every 31st row vs the oracle."""
    import orc
    import rt_hip
    from test_gpu_parity import _mirror_cloud

    monkeypatch.setenv("RT_HIP_DEFER", "1")  # the checked build reads the tuning knobs too
    W, H, D = 512, 384, 6
    text = _mirror_cloud(7, 400)
    sc = rt_hip.Scene.parse(text)
    r = rt_hip.Renderer(0, variant="check")
    try:
        r.upload(sc)
        _, st2 = r.render(sc.camera(), W, H, 2)
        _, st3 = r.render(sc.camera(), W, H, 3)
        assert st3.rays_reflect - st2.rays_reflect > W * H // 8  # more level-2 rays than the queue's room
        rgb, _ = r.render(sc.camera(), W, H, D)
    finally:
        r.close()
    full = np.frombuffer(bytes(rgb), np.uint8).reshape(H, W, 3)
    ref = orc.OracleScene(text=text)
    for y in range(0, H, 31):
        row, _, _ = ref.render(W, H, D, band=1, first=y, stride=1, count=1, threads=8)
        assert full[y].tobytes() == row, f"row {y}"


def test_checked_tiles_and_shards(check_renderer):
    """The one-tile-per-wave global-stack kernels (rt_render_tile into a fp64
    framebuffer) and a row shard with its padding rows."""
    import rt_hip
    import torch

    name = "complex_97x61_d4"
    m = manifest()[name]
    W, H, D = m["width"], m["height"], m["depth"]
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    check_renderer.upload(sc)
    fb = torch.zeros((H * W * 3,), dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    check_renderer.render_tile(sc.camera(), W, H, D, 5, 7, 40, 33, rt_hip.RT_FB_F64X3, fb.data_ptr())
    check_renderer.stats()
    rows = rt_hip.rows_for_shard(H, 8, 1, 3)
    rgb, _ = check_renderer.render(sc.camera(), W, H, D, rows=rows)
    want = np.frombuffer(golden_rgb(name), np.uint8).reshape(H, W, 3)
    got = np.frombuffer(bytes(rgb), np.uint8).reshape(rows.count, W, 3)
    for k in range(rows.count):
        y = (k // 8) * 8 * 3 + 8 + k % 8
        if y < H:
            assert got[k].tobytes() == want[y].tobytes(), f"shard row {k} (image row {y})"


def test_check_library_is_a_test_variant():
    """The product library is not the checked one (its kernels carry no checks)."""
    import rt_hip

    assert os.path.basename(rt_hip.LIB_PATH) == "librt_hip.so"
    assert os.path.exists(rt_hip.VARIANTS["check"])
