"""SURVEY 8(f) rows 2 and 3 on the GPU.

Unquantised framebuffers are compared within MAX_ULP units in the last place:
the specular term uses the device's fp64 `pow` (ocml), which may differ from
glibc's by 1 ulp; everything else in the colour is the
reference's exact operation sequence.  The quantised RGB8 outputs are
compared byte for byte.

* rt_render_tile -- launch_gpu_kernel's tile semantics (src/kernel.cu:185-200,
  99-112): tiles rendered into a full-image device framebuffer reproduce the
  oracle's fp64 framebuffer bit for bit (RT_FB_F64X3, the serial Vec3 fb of
  main.cpp:156), its fp32 rounding (RT_FB_F32X3, the reference's float3 fb)
  and the golden RGB8 image (RT_FB_RGB8), including ragged edge tiles and
  tiles that overhang the image (clipped as kernel.cu:103).
* rt_render_tiles -- a list of such tiles in one launch (the hybrid
  driver's GPU share): the tiles' pixels as rt_render_tile's, only the 8x8
  blocks overlapping them written.
* rt_set_antialias(4) -- the `-a` mode (main_gpu.cu:249-333) in the serial
  fp64 semantics, against the oracle's restatement (orc_render_aa).  The
  reference has no CPU antialias path, so this parity is pinned through the
  oracle's single-sample functions (themselves pinned to the reference's
  golden images), not to a reference fixture.
"""
import numpy as np
import pytest

from conftest import diff_summary, golden_rgb, manifest, scene_path

pytestmark = pytest.mark.gpu


MAX_ULP = 64


def ulp_diff(a, b):
    """Distance in units in the last place between equal-shaped float64 arrays."""
    ia = a.view(np.int64).astype(np.int64)
    ib = b.view(np.int64).astype(np.int64)
    # map the sign-magnitude bit patterns onto a monotone integer line
    ia = np.where(ia < 0, np.int64(-(2**63)) - ia, ia)
    ib = np.where(ib < 0, np.int64(-(2**63)) - ib, ib)
    return np.abs(ia - ib)


def _tiles(W, H, tw, th):
    for ty in range(0, H, th):
        for tx in range(0, W, tw):
            yield tx, ty, tw, th


@pytest.mark.parametrize("tw,th", [(32, 32), (13, 7), (97, 61), (40, 100)])
def test_tiles_f64_match_oracle_framebuffer(gpu_renderer, tw, th):
    import orc
    import rt_hip
    import torch

    name = "complex_97x61_d4"
    m = manifest()[name]
    W, H, D = m["width"], m["height"], m["depth"]
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    gpu_renderer.upload(sc)
    fb = torch.full((H * W * 3,), float("nan"), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()  # the fill (torch's stream) lands before the tiles
    total = 0
    for tx, ty, w, h in _tiles(W, H, tw, th):
        gpu_renderer.render_tile(sc.camera(), W, H, D, tx, ty, w, h, rt_hip.RT_FB_F64X3, fb.data_ptr())
        st = gpu_renderer.stats()
        total += st.rays_primary + st.rays_shadow + st.rays_reflect
    got = fb.cpu().numpy().reshape(H, W, 3)
    _, counts, _, ref_fb = orc.OracleScene(scene_path(m["scene"])).render(W, H, D, threads=4, want_fb=True)
    # oracle fb is in PPM row order; the tile framebuffer is indexed j*W + x with j = 0 the bottom row
    ref = np.array(ref_fb, dtype=np.float64).reshape(H, W, 3)[::-1]
    d = ulp_diff(got, ref)
    assert np.isfinite(got).all()
    assert d.max() <= MAX_ULP, (int(d.max()), int((d > 0).sum()))
    assert total == counts["primary"] + counts["shadow"] + counts["reflect"]


def test_tiles_f32_and_rgb8(gpu_renderer):
    import orc
    import rt_hip
    import torch

    name = "medium_1280x720_d10"
    m = manifest()[name]
    W, H, D = m["width"], m["height"], m["depth"]
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    gpu_renderer.upload(sc)
    f32 = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    rgb = torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill (torch's stream) lands before the tiles
    for tx, ty, w, h in _tiles(W, H, 200, 150):  # ragged right and top edges
        gpu_renderer.render_tile(sc.camera(), W, H, D, tx, ty, w, h, rt_hip.RT_FB_F32X3, f32.data_ptr())
        gpu_renderer.render_tile(sc.camera(), W, H, D, tx, ty, w, h, rt_hip.RT_FB_RGB8, rgb.data_ptr())
    gpu_renderer.stats()
    assert rgb.cpu().numpy().tobytes() == golden_rgb(name)
    _, _, _, ref_fb = orc.OracleScene(scene_path(m["scene"])).render(W, H, D, threads=8, want_fb=True)
    ref = np.array(ref_fb, dtype=np.float64).reshape(H, W, 3)[::-1]
    got = f32.cpu().numpy().reshape(H, W, 3).astype(np.float64)
    # float(x) of values within MAX_ULP fp64 ulps: equal or one float ulp apart
    err = np.abs(got - ref) - (np.abs(ref) * 2.0**-23 + 2.0**-125)  # float denormals lose relative precision
    assert (err <= 0).all(), (float(err.max()), np.argwhere(err > 0)[:3].tolist())


def test_tile_leaves_other_pixels_alone(gpu_renderer):
    import rt_hip
    import torch

    W, H, D = 64, 48, 3
    sc = rt_hip.Scene.load(scene_path("complex"))
    gpu_renderer.upload(sc)
    fb = torch.full((H * W * 3,), 7, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill (torch's stream) lands before the tiles
    gpu_renderer.render_tile(sc.camera(), W, H, D, 10, 5, 20, 9, rt_hip.RT_FB_RGB8, fb.data_ptr())
    st = gpu_renderer.stats()
    assert st.rays_primary == 20 * 9
    img = fb.cpu().numpy().reshape(H, W, 3)
    mask = np.zeros((H, W), bool)
    mask[H - 5 - 9:H - 5, 10:30] = True  # bottom-up rows 5..13 are PPM rows H-14..H-6
    assert (img[~mask] == 7).all()
    # overhanging and empty tiles are clipped
    gpu_renderer.render_tile(sc.camera(), W, H, D, 60, 40, 100, 100, rt_hip.RT_FB_RGB8, fb.data_ptr())
    assert gpu_renderer.stats().rays_primary == 4 * 8
    gpu_renderer.render_tile(sc.camera(), W, H, D, 70, 0, 5, 5, rt_hip.RT_FB_RGB8, fb.data_ptr())
    assert gpu_renderer.stats().rays_primary == 0
    with pytest.raises(rt_hip.RtError):
        gpu_renderer.render_tile(sc.camera(), W, H, D, 0, 0, 8, 8, 9, fb.data_ptr())


@pytest.mark.parametrize("tiles", [
    [(0, 0, 32, 32), (40, 13, 17, 9), (90, 50, 100, 100)],      # ragged, overhanging
    [(tx, ty, 13, 7) for tx, ty, _, _ in _tiles(97, 61, 13, 7)],  # every pixel, unaligned tiles
    [(5, 5, 3, 3), (5, 5, 3, 3), (6, 6, 30, 2)],                  # duplicated and overlapping
])
def test_tiles_batch_match_oracle_framebuffer(gpu_renderer, tiles):
    """rt_render_tiles: the listed tiles' pixels in ONE launch equal rt_render_tile's
    (the oracle's fp64 framebuffer within MAX_ULP); only the 8x8 blocks that
    overlap a tile are written."""
    import orc
    import rt_hip
    import torch

    name = "complex_97x61_d4"
    m = manifest()[name]
    W, H, D = m["width"], m["height"], m["depth"]
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    gpu_renderer.upload(sc)
    fb = torch.full((H * W * 3,), float("nan"), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()  # the fill (torch's stream) lands before the launch
    gpu_renderer.render_tiles(sc.camera(), W, H, D, tiles, rt_hip.RT_FB_F64X3, fb.data_ptr())
    gpu_renderer.stats()
    got = fb.cpu().numpy().reshape(H, W, 3)
    _, _, _, ref_fb = orc.OracleScene(scene_path(m["scene"])).render(W, H, D, threads=4, want_fb=True)
    ref = np.array(ref_fb, dtype=np.float64).reshape(H, W, 3)[::-1]  # index j*W + x, j = 0 the bottom row
    want = np.zeros((H, W), bool)  # the tiles' pixels
    blocks = np.zeros((H, W), bool)  # the 8x8 blocks (PPM row order) that overlap a tile
    for x, y, w, h in tiles:
        x1, j1 = min(W, x + w), min(H, y + h)
        if x >= x1 or y >= j1:
            continue
        want[y:j1, x:x1] = True
        p0, p1 = H - j1, H - 1 - y  # PPM rows of the tile
        for by in range(p0 // 8, p1 // 8 + 1):
            for bx in range(x // 8, (x1 - 1) // 8 + 1):
                r0, r1 = by * 8, min(H, by * 8 + 8)  # PPM rows -> framebuffer rows j = H-1-row
                blocks[H - r1:H - r0, bx * 8:min(W, bx * 8 + 8)] = True
    assert ulp_diff(got[want], ref[want]).max() <= MAX_ULP
    assert np.isfinite(got[blocks]).all()
    assert np.isnan(got[~blocks]).all()


def test_tiles_batch_rgb8_and_errors(gpu_renderer):
    import rt_hip
    import torch

    name = "medium_1280x720_d10"
    m = manifest()[name]
    W, H, D = m["width"], m["height"], m["depth"]
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    gpu_renderer.upload(sc)
    rgb = torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    gpu_renderer.render_tiles(sc.camera(), W, H, D, list(_tiles(W, H, 64, 64)), rt_hip.RT_FB_RGB8, rgb.data_ptr())
    st = gpu_renderer.stats()
    assert rgb.cpu().numpy().tobytes() == golden_rgb(name)
    assert st.rays_primary == W * H
    gpu_renderer.render_tiles(sc.camera(), W, H, D, [], rt_hip.RT_FB_RGB8, rgb.data_ptr())  # nothing to do
    assert gpu_renderer.stats().rays_primary == 0
    for bad in ([(0, 0, -1, 4)], [(-3, 0, 4, 4)]):
        with pytest.raises(rt_hip.RtError):
            gpu_renderer.render_tiles(sc.camera(), W, H, D, bad, rt_hip.RT_FB_RGB8, rgb.data_ptr())
    with pytest.raises(rt_hip.RtError):
        gpu_renderer.render_tiles(sc.camera(), W, H, D, [(0, 0, 8, 8)], 9, rgb.data_ptr())


@pytest.fixture
def aa_renderer(gpu_renderer):
    gpu_renderer.set_antialias(4)
    yield gpu_renderer
    gpu_renderer.set_antialias(1)


@pytest.mark.parametrize("scene,W,H,D", [("complex", 97, 61, 4), ("medium", 160, 90, 5), ("simple", 64, 48, 10),
                                         ("synth200", 120, 68, 4)])
def test_antialias_matches_oracle(aa_renderer, scene, W, H, D):
    import orc
    import rt_hip

    sc = rt_hip.Scene.load(scene_path(scene))
    aa_renderer.upload(sc)
    rgb, st = aa_renderer.render(sc.camera(), W, H, D)
    ref, counts, _ = orc.OracleScene(scene_path(scene)).render_aa(W, H, D, samples=4, threads=4)
    assert bytes(rgb) == ref, diff_summary(bytes(rgb), ref)
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (counts["primary"], counts["shadow"],
                                                                   counts["reflect"])
    assert st.rays_primary == 4 * W * H


def test_antialias_tiles_and_deep_depth(aa_renderer):
    import orc
    import rt_hip
    import torch

    W, H, D = 50, 40, 9  # depth > 5 takes the persistent kernel
    sc = rt_hip.Scene.load(scene_path("complex"))
    aa_renderer.upload(sc)
    fb = torch.zeros(H * W * 3, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()  # the fill (torch's stream) lands before the tiles
    for tx, ty, w, h in _tiles(W, H, 16, 16):
        aa_renderer.render_tile(sc.camera(), W, H, D, tx, ty, w, h, rt_hip.RT_FB_F64X3, fb.data_ptr())
    aa_renderer.stats()
    _, _, _, ref_fb = orc.OracleScene(scene_path("complex")).render_aa(W, H, D, samples=4, threads=4, want_fb=True)
    ref = np.array(ref_fb, dtype=np.float64).reshape(H, W, 3)[::-1]
    assert ulp_diff(fb.cpu().numpy().reshape(H, W, 3), ref).max() <= MAX_ULP
    rgb, _ = aa_renderer.render(sc.camera(), W, H, D)
    ref8, _, _ = orc.OracleScene(scene_path("complex")).render_aa(W, H, D, samples=4, threads=4)
    assert bytes(rgb) == ref8


def test_antialias_setter_rejects_other_counts(gpu_renderer):
    import rt_hip

    for bad in (0, 2, 3, 8):
        with pytest.raises(rt_hip.RtError):
            gpu_renderer.set_antialias(bad)
