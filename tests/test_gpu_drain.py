"""GPU: drain mode (tuning build, RT_HIP_DRAIN): the merged kernel's waves run
the launch's deferred reflection rays themselves once their own tiles are
done -- no render_deferred launch.  Deferred entries are tagged per launch and
kept per XCD; a tile's flush leaves its deferred pixels' bytes to the rays
that finish them (store_row_dword / put_px).  Every image must equal the
reference's (goldens) or the oracle, with the same ray counts as the
two-kernel path."""
import numpy as np
import pytest

from conftest import diff_summary, golden_rgb, knob_variant, manifest, scene_path

pytestmark = pytest.mark.gpu


def _renderer(monkeypatch, drain, defer=None):
    import rt_hip

    monkeypatch.setenv("RT_HIP_DRAIN", str(drain))
    if defer is not None:
        monkeypatch.setenv("RT_HIP_DEFER", str(defer))
    return rt_hip.Renderer(0, variant=knob_variant())


def _frames(r, cams, W, H, D, rows=None):
    import torch

    R = rows.count if rows is not None else H
    stride = R * W * 3
    buf = torch.full((len(cams) * stride,), 77, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    r.render_frames_async(cams, W, H, D, rows, buf.data_ptr(), stride)
    st = r.stats()
    host = buf.cpu().numpy()
    return [host[f * stride:(f + 1) * stride] for f in range(len(cams))], st


@pytest.mark.parametrize("name", sorted(manifest()))
def test_drain_one_frame_goldens(monkeypatch, name):
    """Every golden, one-frame launches deferring (RT_HIP_DRAIN=2)."""
    import rt_hip

    r = _renderer(monkeypatch, 2)
    try:
        m = manifest()[name]
        sc = rt_hip.Scene.load(scene_path(m["scene"]))
        r.upload(sc)
        rgb, st = r.render(sc.camera(), m["width"], m["height"], m["depth"])
        want = golden_rgb(name)
        assert bytes(rgb) == want, diff_summary(bytes(rgb), want)
        rays = m["rays"]
        assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (rays["primary"], rays["shadow"], rays["reflect"])
        if m["depth"] > 2 and m["width"] * m["height"] >= 1024:
            assert r.info().deferred_last == 2
    finally:
        r.close()


@pytest.mark.parametrize("F", [2, 20, 32])
def test_drain_multi_frame_golden(monkeypatch, F):
    """The bench's launch shapes on the metric workload with drain mode 1."""
    import rt_hip

    r = _renderer(monkeypatch, 1)
    try:
        name = "synth200_1920x1080_d4"
        m = manifest()[name]
        sc = rt_hip.Scene.load(scene_path(m["scene"]))
        r.upload(sc)
        want = golden_rgb(name)
        for _ in range(2):  # the second launch reuses the queue: entries of the first carry another tag
            frames, st = _frames(r, [sc.camera()] * F, m["width"], m["height"], m["depth"])
            assert r.info().deferred_last == 2
            for f in range(F):
                assert frames[f].tobytes() == want, f"frame {f}: {diff_summary(frames[f].tobytes(), want)}"
            rays = m["rays"]
            assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (F * rays["primary"], F * rays["shadow"],
                                                                           F * rays["reflect"])
    finally:
        r.close()


def test_drain_row_shard_and_odd_width(monkeypatch):
    """Tiles that are not whole (odd width: put_px for every pixel, deferred
    ones skipped by the flush) and a row shard with padding rows."""
    import orc
    import rt_hip

    r = _renderer(monkeypatch, 2)
    try:
        name = "complex_97x61_d4"
        m = manifest()[name]
        W, H, D = m["width"], m["height"], m["depth"]
        sc = rt_hip.Scene.load(scene_path(m["scene"]))
        r.upload(sc)
        rgb, _ = r.render(sc.camera(), W, H, D)
        assert bytes(rgb) == golden_rgb(name)
        rows = rt_hip.rows_for_shard(H, 8, 1, 3)
        got, _ = r.render(sc.camera(), W, H, D, rows=rows)
        want = np.frombuffer(golden_rgb(name), np.uint8).reshape(H, W, 3)
        got = np.frombuffer(bytes(got), np.uint8).reshape(rows.count, W, 3)
        for k in range(rows.count):
            y = (k // 8) * 8 * 3 + 8 + k % 8
            if y < H:
                assert got[k].tobytes() == want[y].tobytes(), f"shard row {k} (image row {y})"
        text = open(scene_path("complex")).read()
        W2, H2 = 203, 97
        rgb2, _ = r.render(sc.camera(), W2, H2, 5)
        ref, _, _ = orc.OracleScene(text=text).render(W2, H2, 5, threads=8)
        assert bytes(rgb2) == ref, diff_summary(bytes(rgb2), ref)
    finally:
        r.close()


@pytest.mark.parametrize("n", [400, 1300])
def test_drain_queue_overflow_vs_oracle(monkeypatch, n):
    """A camera inside a mirror cloud: more level-2 rays than the queue holds
    (the rest stay in their lanes); drain-mode image and ray counts equal the
    render without deferral; every 31st row equals the oracle's."""
    import orc
    import rt_hip
    from test_gpu_parity import _mirror_cloud

    W, H, D = 512, 384, 6
    text = _mirror_cloud(7, n)
    sc = rt_hip.Scene.parse(text)
    r = _renderer(monkeypatch, 2)
    try:
        r.upload(sc)
        rgb, st = r.render(sc.camera(), W, H, D)
        assert r.info().deferred_last == 2
    finally:
        r.close()
    r0 = _renderer(monkeypatch, 0, defer=0)
    try:
        r0.upload(sc)
        rgb0, st0 = r0.render(sc.camera(), W, H, D)
    finally:
        r0.close()
    assert bytes(rgb) == bytes(rgb0), diff_summary(bytes(rgb), bytes(rgb0))
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (st0.rays_primary, st0.rays_shadow, st0.rays_reflect)
    full = np.frombuffer(bytes(rgb), np.uint8).reshape(H, W, 3)
    ref = orc.OracleScene(text=text)
    for y in range(0, H, 31):
        row, _, _ = ref.render(W, H, D, band=1, first=y, stride=1, count=1, threads=8)
        assert full[y].tobytes() == row, f"row {y}"


def test_drain_cfg5_rows(monkeypatch):
    """synth10k 384x216 d6 (uniform-grid walks, deep chains) as a 3-frame
    drain launch against its golden."""
    import rt_hip

    r = _renderer(monkeypatch, 1)
    try:
        name = "synth10k_384x216_d6"
        m = manifest()[name]
        sc = rt_hip.Scene.load(scene_path(m["scene"]))
        r.upload(sc)
        frames, _ = _frames(r, [sc.camera()] * 3, m["width"], m["height"], m["depth"])
        for f in range(3):
            assert frames[f].tobytes() == golden_rgb(name), f
    finally:
        r.close()
