"""GPU parity: the HIP render loop against the reference's golden images and the
CPU oracle, through the C-ABI (librt_hip.so).  Bar: byte-identical RGB8 and
identical ray counts (the north star allows +-1 per channel; the fp64 kernel
is held to exact equality, and the +-1 bound is asserted separately so a
failure report shows both)."""
import numpy as np
import pytest

from conftest import diff_summary, golden_rgb, manifest, scene_path, knob_variant

pytestmark = pytest.mark.gpu

GOLDEN_NAMES = sorted(manifest().keys())


def _render(r, name, rows=None):
    import rt_hip

    m = manifest()[name]
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    r.upload(sc)
    rgb, st = r.render(sc.camera(), m["width"], m["height"], m["depth"], rows=rows)
    return bytes(rgb), st, m


@pytest.fixture(params=[True, False], ids=["cull", "brute"])
def culling(request, gpu_renderer):
    gpu_renderer.set_culling(request.param)
    yield request.param
    gpu_renderer.set_culling(True)


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_golden_byte_identical(gpu_renderer, culling, name):
    rgb, st, m = _render(gpu_renderer, name)
    want = golden_rgb(name)
    d = np.abs(np.frombuffer(rgb, np.uint8).astype(int) - np.frombuffer(want, np.uint8).astype(int))
    assert d.max(initial=0) <= 1, f"{name}: beyond +-1/255: {diff_summary(rgb, want)}"
    assert rgb == want, f"{name}: {diff_summary(rgb, want)}"


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_ray_counts_match_oracle(gpu_renderer, name):
    _, st, m = _render(gpu_renderer, name)
    assert {"primary": st.rays_primary, "shadow": st.rays_shadow, "reflect": st.rays_reflect} == m["rays"]
    assert st.negative_clamped == 0


@pytest.mark.parametrize("G,band", [(2, 8), (3, 8), (8, 8), (5, 1), (4, 16)])
def test_row_shards_reassemble(gpu_renderer, G, band):
    """Cyclic row bands rendered separately and unpermuted equal the full frame."""
    import rt_hip

    name = "complex_97x61_d4"
    m = manifest()[name]
    want = golden_rgb(name)
    W, H = m["width"], m["height"]
    shards = []
    total = {"primary": 0, "shadow": 0, "reflect": 0}
    for r in range(G):
        rows = rt_hip.rows_for_shard(H, band, r, G)
        rgb, st, _ = _render(gpu_renderer, name, rows)
        shards.append(np.frombuffer(rgb, np.uint8).reshape(rows.count, W, 3))
        total["primary"] += st.rays_primary
        total["shadow"] += st.rays_shadow
        total["reflect"] += st.rays_reflect
    R = shards[0].shape[0]
    img = np.zeros((H, W, 3), np.uint8)
    for y in range(H):
        b = y // band
        img[y] = shards[b % G][(b // G) * band + y % band]
    assert img.tobytes() == want
    assert total == m["rays"]
    # padding rows are zero-filled
    for r in range(G):
        rows = rt_hip.rows_for_shard(H, band, r, G)
        for k in range(R):
            y = (k // band) * band * G + r * band + k % band
            if y >= H:
                assert not shards[r][k].any()


def test_unpermute_kernel(gpu_renderer):
    import torch
    import rt_hip

    name = "complex_97x61_d4"
    m = manifest()[name]
    W, H, G, band = m["width"], m["height"], 3, 8
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    gpu_renderer.upload(sc)
    R = rt_hip.rows_for_shard(H, band, 0, G).count
    gathered = torch.zeros((G, R, W, 3), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()  # the zero-fill (torch's stream) lands before the renders
    for r in range(G):
        gpu_renderer.render(sc.camera(), W, H, m["depth"], rows=rt_hip.rows_for_shard(H, band, r, G),
                            out=gathered[r], out_on_device=True)
    image = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
    gpu_renderer.unpermute(gathered.data_ptr(), image.data_ptr(), W, H, band, G, R)
    gpu_renderer.stats()  # synchronises the context stream
    assert image.cpu().numpy().tobytes() == golden_rgb(name)


@pytest.mark.parametrize("W,G,band,off", [(1920, 8, 8, 0), (100, 3, 8, 0), (100, 3, 8, 4), (64, 5, 1, 1),
                                          (97, 2, 16, 0)])
def test_unpermute_copy_widths(gpu_renderer, W, G, band, off):
    """The unpermute's 16-byte, 4-byte and byte copy paths (row bytes W*3 and
    buffer offsets decide which) against the host permutation."""
    import torch

    H = 75
    R = -(-(-(-H // band)) // G) * band
    src = torch.randint(0, 256, (off + G * R * W * 3,), dtype=torch.uint8, device="cuda:0")
    dst = torch.zeros((off + H * W * 3,), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()  # both fills (torch's stream) land before the unpermute
    gpu_renderer.unpermute(src.data_ptr() + off, dst.data_ptr() + off, W, H, band, G, R)
    gpu_renderer.stats()
    s = src[off:].cpu().numpy().reshape(G, R, W * 3)
    want = np.stack([s[(y // band) % G][(y // band // G) * band + y % band] for y in range(H)])
    assert dst[off:].cpu().numpy().reshape(H, W * 3).tobytes() == want.tobytes()


def test_async_on_external_stream(gpu_renderer):
    import torch
    import rt_hip

    name = "simple_800x600_d10"
    m = manifest()[name]
    sc = rt_hip.Scene.load(scene_path(m["scene"]))
    gpu_renderer.upload(sc)
    out = torch.empty((m["height"], m["width"], 3), dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.Stream()
    gpu_renderer.set_stream(s.cuda_stream)
    try:
        gpu_renderer.render_async(sc.camera(), m["width"], m["height"], m["depth"], None, out.data_ptr())
        st = gpu_renderer.stats()
    finally:
        gpu_renderer.set_stream(None)
    assert out.cpu().numpy().tobytes() == golden_rgb(name)
    assert st.kernel_ms > 0


@pytest.mark.parametrize("depth", [0, 1, 2, 5, 17, 64])
def test_depth_edges_vs_oracle(gpu_renderer, depth):
    import orc
    import rt_hip

    W, H = 67, 45
    sc = rt_hip.Scene.load(scene_path("medium"))
    gpu_renderer.upload(sc)
    rgb, st = gpu_renderer.render(sc.camera(), W, H, depth)
    ref, counts, _ = orc.OracleScene(scene_path("medium")).render(W, H, depth, threads=4)
    assert bytes(rgb) == ref, diff_summary(bytes(rgb), ref)
    assert st.rays_primary == counts["primary"] and st.rays_shadow == counts["shadow"]
    assert st.rays_reflect == counts["reflect"]


def test_depth_limit_is_an_error(gpu_renderer):
    import rt_hip

    sc = rt_hip.Scene.load(scene_path("simple"))
    gpu_renderer.upload(sc)
    with pytest.raises(rt_hip.RtError) as e:
        gpu_renderer.render(sc.camera(), 8, 8, rt_hip.RT_MAX_DEPTH + 1)
    assert e.value.status == 7


MIRRORS = """
# two facing mirrors: a reflection chain as long as the depth allows
sphere 0 0 -6 2 0.9 0.9 0.9 1.0 0.5 50
sphere 0 0 6 2 0.9 0.9 0.9 1.0 0.5 50
sphere 4 0 0 1 0.2 0.8 0.2 0.5 0.5 20
light 0 10 0 1 1 1 1
light 0 0 0 0.5 0.5 0.5 1
ambient 0.2 0.2 0.2
camera 0 0.3 0 0 0 -6 90
"""

EDGE_SCENES = {
    "empty": "camera 0 0 0 0 0 -1 60\n",  # no spheres, no lights: all sky
    "no_lights": "sphere 0 0 -5 1 1 0 0 0.5 1 10\nambient 0.3 0.3 0.3\n",
    "no_camera": "sphere 0 0 -5 1 1 0 0 0 1 10\nlight 5 5 0 1 1 1 1\n",  # default camera scene.h:22
    "mirrors": MIRRORS,
    "inside_sphere": "sphere 0 0 0 5 0.5 0.5 0.5 0.5 1 10\nlight 0 0 0 1 1 1 1\ncamera 0 0 0 0 0 -1 60\n",
    "tangent": "sphere 1 0 -5 1 1 1 1 0 1 1\nsphere -1 0 -5 1 1 0 1 0.3 1 3\nlight 0 0 10 1 1 1 1\n"
               "camera 0 0 0 0 0 -5 60\n",
    "shininess_zero": "sphere 0 0 -5 1 1 1 1 0 1 0\nlight 0 3 0 1 1 1 1\nambient 0.1 0.1 0.1\n",
    "bright": "sphere 0 0 -5 1 4 4 4 0 1 2\nlight 0 3 0 3 3 3 1\nambient 2 2 2\n",  # saturating channels
}


@pytest.mark.parametrize("name", sorted(EDGE_SCENES))
@pytest.mark.parametrize("depth", [1, 4, 10])
def test_edge_scenes_vs_oracle(gpu_renderer, name, depth):
    import orc
    import rt_hip

    W, H = 64, 48
    sc = rt_hip.Scene.parse(EDGE_SCENES[name])
    gpu_renderer.upload(sc)
    rgb, st = gpu_renderer.render(sc.camera(), W, H, depth)
    ref, counts, _ = orc.OracleScene(text=EDGE_SCENES[name]).render(W, H, depth, threads=2)
    assert bytes(rgb) == ref, diff_summary(bytes(rgb), ref)
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (counts["primary"], counts["shadow"],
                                                                   counts["reflect"])


def test_4k_shards_match_sampled_oracle_rows(gpu_renderer):
    """BASELINE cfg 4 (complex 3840x2160 d4), 8 cyclic shards: every 97th output row
    equals the oracle's, and per-shard ray counts sum to the full-frame counts."""
    import orc
    import rt_hip

    W, H, D, G, band = 3840, 2160, 4, 8, 8
    sc = rt_hip.Scene.load(scene_path("complex"))
    gpu_renderer.upload(sc)
    full, st_full = gpu_renderer.render(sc.camera(), W, H, D)
    full = np.frombuffer(bytes(full), np.uint8).reshape(H, W, 3)
    tot = 0
    img = np.zeros_like(full)
    for r in range(G):
        rows = rt_hip.rows_for_shard(H, band, r, G)
        rgb, st = gpu_renderer.render(sc.camera(), W, H, D, rows=rows)
        sh = np.frombuffer(bytes(rgb), np.uint8).reshape(rows.count, W, 3)
        for k in range(rows.count):
            y = (k // band) * band * G + r * band + k % band
            if y < H:
                img[y] = sh[k]
        tot += st.rays
    assert np.array_equal(img, full)
    assert tot == st_full.rays
    ref = orc.OracleScene(scene_path("complex"))
    for y in range(0, H, 97):
        rgb, _, _ = ref.render(W, H, D, band=1, first=y, stride=1, count=1)
        assert full[y].tobytes() == rgb, f"row {y}"


FRAC_SHININESS = (0.5, 7.5, 33.3, 1500.25)


def _shininess(rng, frac: bool) -> str:
    """Whole shininess (int_pow), or fractional (dd_pow: scene.h:113's pow off
    the integers): fixed values and uniform draws in [0.5, 2000)."""
    if not frac:
        return "%d" % rng.choice([1, 5, 20, 100])
    return "%.3f" % (rng.choice(FRAC_SHININESS) if rng.random() < 0.5 else rng.uniform(0.5, 2000.0))


def _random_scene(seed: int, n: int, frac: bool = False) -> str:
    """Dense random scenes: tiny and huge spheres, spheres behind and around the
    camera, the camera inside a sphere for some seeds, many lights."""
    import random

    rng = random.Random(seed)
    lines = []
    for _ in range(n):
        r = rng.choice([0.01, 0.05, 0.2, 0.5, 1.0, 3.0]) * rng.uniform(0.5, 1.5)
        lines.append("sphere %.6f %.6f %.6f %.6f %.3f %.3f %.3f %.2f 0.5 %s" % (
            rng.uniform(-12, 12), rng.uniform(-8, 8), rng.uniform(-40, 10), r, rng.random(), rng.random(),
            rng.random(), rng.choice([0.0, 0.0, 0.3, 0.7, 1.0]), _shininess(rng, frac)))
    for _ in range(rng.randint(1, 6)):
        lines.append("light %.3f %.3f %.3f %.3f %.3f %.3f 1" % (rng.uniform(-15, 15), rng.uniform(-5, 15),
                                                               rng.uniform(-30, 10), rng.random(), rng.random(),
                                                               rng.random()))
    lines.append("ambient 0.1 0.1 0.1")
    cz = rng.choice([5.0, 0.0, -10.0])
    lines.append("camera %.3f %.3f %.3f 0 0 -20 %d" % (rng.uniform(-2, 2), rng.uniform(-1, 3), cz,
                                                      rng.choice([30, 65, 120])))
    return "\n".join(lines) + "\n"


@pytest.mark.parametrize("seed", range(12))
def test_random_dense_scenes_vs_oracle(gpu_renderer, seed):
    import orc
    import rt_hip

    text = _random_scene(seed, 60 + 40 * seed)
    W, H, D = 96, 64, 5
    sc = rt_hip.Scene.parse(text)
    gpu_renderer.upload(sc)
    ref, counts, _ = orc.OracleScene(text=text).render(W, H, D, threads=4)
    for cull in (True, False):
        gpu_renderer.set_culling(cull)
        rgb, st = gpu_renderer.render(sc.camera(), W, H, D)
        assert bytes(rgb) == ref, (cull, diff_summary(bytes(rgb), ref))
        assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (counts["primary"], counts["shadow"],
                                                                       counts["reflect"])
    gpu_renderer.set_culling(True)


def _pm1(got: bytes, want: bytes):
    """The north star's bar: every channel within 1 of the oracle's; returns the
    number of differing channels (expected 0: the kernel is exact where the pow
    agrees with glibc's, and a 1-ulp pow difference moves a byte only next to a
    quantisation boundary)."""
    d = np.abs(np.frombuffer(got, np.uint8).astype(np.int16) - np.frombuffer(want, np.uint8).astype(np.int16))
    assert d.size and int(d.max()) <= 1, diff_summary(got, want)
    return int((d > 0).sum())


@pytest.mark.parametrize("seed", range(8))
def test_fractional_shininess_scenes_vs_oracle(gpu_renderer, seed):
    """Dense random scenes whose shininess is fractional (0.5, 7.5, 33.3,
    1500.25 and uniform draws in [0.5, 2000)): pow(rdv, shininess) is dd_pow
    (rt_pow.h), the oracle's is glibc's.  Bar: +-1 per channel and identical ray
    counts; the number of differing channels is printed (measured: 0)."""
    import orc
    import rt_hip

    text = _random_scene(1000 + seed, 60 + 40 * seed, frac=True)
    W, H, D = 96, 64, 5
    sc = rt_hip.Scene.parse(text)
    gpu_renderer.upload(sc)
    ref, counts, _ = orc.OracleScene(text=text).render(W, H, D, threads=4)
    rgb, st = gpu_renderer.render(sc.camera(), W, H, D)
    nd = _pm1(bytes(rgb), ref)
    print(f"fractional shininess, seed {seed}: {nd} of {len(ref)} channels differ")
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (counts["primary"], counts["shadow"],
                                                                   counts["reflect"])


@pytest.mark.parametrize("n", [400, 1300], ids=["render_deferred", "render_deferred_walk"])
def test_fractional_shininess_mirror_cloud_vs_oracle(monkeypatch, n):
    """A camera inside a cloud of mirrors with fractional shininess: every
    reflection level (merged megakernel, render_deferred / render_deferred_walk:
    RT_HIP_DEFER=1 defers in this one-frame render too) shades with dd_pow.
    +-1 per channel, identical ray counts."""
    import orc
    import rt_hip

    W, H, D = 192, 144, 6
    text = _mirror_cloud(11, n, frac=True)
    sc = rt_hip.Scene.parse(text)
    monkeypatch.setenv("RT_HIP_DEFER", "1")
    r = rt_hip.Renderer(0, variant=knob_variant())
    r.upload(sc)
    ref, counts, _ = orc.OracleScene(text=text).render(W, H, D, threads=8)
    try:
        rgb, st = r.render(sc.camera(), W, H, D)
    finally:
        r.close()
    nd = _pm1(bytes(rgb), ref)
    print(f"fractional shininess mirror cloud n={n}: {nd} of {len(ref)} channels differ")
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (counts["primary"], counts["shadow"],
                                                                   counts["reflect"])


def test_cull_equals_bruteforce_at_4k(gpu_renderer):
    import rt_hip

    sc = rt_hip.Scene.load(scene_path("synth200"))
    gpu_renderer.upload(sc)
    a, sa = gpu_renderer.render(sc.camera(), 3840, 2160, 6)
    gpu_renderer.set_culling(False)
    try:
        b, sb = gpu_renderer.render(sc.camera(), 3840, 2160, 6)
    finally:
        gpu_renderer.set_culling(True)
    assert bytes(a) == bytes(b)
    assert sa.rays == sb.rays


@pytest.fixture(params=[{"RT_HIP_BVH_ALWAYS": "1"}, {"RT_HIP_BVH_ALWAYS": "1", "RT_HIP_BVH4": "0"}],
                ids=["bvh-always", "bvh-always-two-child"])
def bvh_renderer(request, monkeypatch):
    """A fresh context per BVH policy (the knobs are read at rt_create)."""
    import rt_hip

    for k, v in request.param.items():
        monkeypatch.setenv(k, v)
    r = rt_hip.Renderer(0, variant=knob_variant())
    yield r
    r.close()


@pytest.mark.parametrize("name", ["complex_97x61_d4", "medium_1280x720_d10", "synth200_1920x1080_d4",
                                  "synth10k_384x216_d6", "simple_1x1_d10"])
def test_bvh_policies_golden(bvh_renderer, name):
    rgb, st, m = _render(bvh_renderer, name)
    assert rgb == golden_rgb(name), diff_summary(rgb, golden_rgb(name))
    assert {"primary": st.rays_primary, "shadow": st.rays_shadow, "reflect": st.rays_reflect} == m["rays"]


@pytest.mark.parametrize("seed", range(0, 12, 3))
def test_bvh_policies_random_scenes(bvh_renderer, seed):
    import orc
    import rt_hip

    text = _random_scene(seed, 60 + 40 * seed)
    W, H, D = 96, 64, 5
    sc = rt_hip.Scene.parse(text)
    bvh_renderer.upload(sc)
    ref, counts, _ = orc.OracleScene(text=text).render(W, H, D, threads=4)
    rgb, st = bvh_renderer.render(sc.camera(), W, H, D)
    assert bytes(rgb) == ref, diff_summary(bytes(rgb), ref)


def test_bvh_far_from_origin(bvh_renderer):
    """Scene translated far from the origin: the fp32 BVH works relative to the scene centre."""
    import orc
    import rt_hip

    lines = []
    for i in range(40):
        lines.append("sphere %d %d %d 0.7 0.5 0.5 0.9 0.3 0.5 20" % (100000 + (i % 7) * 2, 100000 + (i // 7),
                                                                     -100020 - (i % 5) * 3))
    lines += ["light 100010 100020 -100000 1 1 1 1", "light 99990 100010 -100005 0.5 0.6 0.7 1",
              "camera 100004 100003 -99990 100004 100003 -100020 50"]
    text = "\n".join(lines) + "\n"
    sc = rt_hip.Scene.parse(text)
    bvh_renderer.upload(sc)
    ref, _, _ = orc.OracleScene(text=text).render(80, 60, 6, threads=4)
    rgb, _ = bvh_renderer.render(sc.camera(), 80, 60, 6)
    assert bytes(rgb) == ref, diff_summary(bytes(rgb), ref)


@pytest.mark.parametrize("offset,bounded", [(0, 1), (100000, 1), (100000000, 0)])
def test_shadow_line_check_paths(offset, bounded):
    """shadow_cells skips its per-ray check that a shadow line passes within
    the light grid's margin of its light when the host bounds it for the whole
    scene (rt_info.shadow_line_bounded: 2^-41 (1.01 B + 0.01) <= 1e-7 x the
    scene diameter, B the box's largest |coordinate|).  A scene at the origin
    and 1e5 away takes the bounded path, 1e8 away (B / diameter ~ 3e6) the
    checked one; both against the oracle (scene.h:65-86), image and shadow
    ray count."""
    import orc
    import rt_hip

    lines = []
    for i in range(40):
        lines.append("sphere %d %d %d 0.7 0.5 0.5 0.9 0.3 0.5 20" % (offset + (i % 7) * 2, offset + (i // 7),
                                                                     -offset - 20 - (i % 5) * 3))
    lines += ["light %d %d %d 1 1 1 1" % (offset + 10, offset + 20, -offset),
              "light %d %d %d 0.5 0.6 0.7 1" % (offset - 10, offset + 10, -offset - 5),
              "camera %d %d %d %d %d %d 50" % (offset + 4, offset + 3, -offset + 10, offset + 4, offset + 3,
                                              -offset - 20)]
    text = "\n".join(lines) + "\n"
    sc = rt_hip.Scene.parse(text)
    r = rt_hip.Renderer(0)
    try:
        r.upload(sc)
        assert r.info().shadow_line_bounded == bounded
        W, H, D = 96, 64, 6
        ref, counts, _ = orc.OracleScene(text=text).render(W, H, D, threads=4)
        rgb, st = r.render(sc.camera(), W, H, D)
        assert bytes(rgb) == ref, diff_summary(bytes(rgb), ref)
        assert st.rays_shadow == counts["shadow"]
    finally:
        r.close()


# the layouts the product reaches without a knob (the global stack: tiles,
# antialias; scanline order: launches under 1,024 tiles; an 8-entry merge
# queue: scenes whose walk stacks fill the LDS; deferral on / off: multi- /
# one-frame launches) plus the north star's LDS-staged scene
@pytest.fixture(params=[{"RT_HIP_LDS_SCENE": "1"}, {"RT_HIP_SCHED": "0"}, {"RT_HIP_STACK": "1"},
                        {"RT_HIP_DEFER": "0"}, {"RT_HIP_DEFER": "1"}, {"RT_HIP_MERGE_Q": "8"}],
                ids=["lds-scene", "scanline-order", "global-stack", "no-defer", "defer-one-frame",
                     "merge-queue-8"])
def stack_renderer(request, monkeypatch):
    """Non-default kernel layouts (RT_HIP_STACK=1: one tile per wave with the
    per-pixel global stack instead of merged levels; RT_HIP_LDS_SCENE=1:
    scenes that fit staged in LDS with 4-wave workgroups; RT_HIP_SCHED=0: tiles
    launched in scanline order instead of heaviest-predicted first;
    RT_HIP_MERGE_Q / RT_HIP_DEFER: merge-queue size and the deferred-ray kernel
    (these single-frame renders defer only with RT_HIP_DEFER=1: by default
    one-frame launches keep every level in the megakernel)).  Knobs other
    than RT_HIP_LDS_SCENE are read by the tuning build only."""
    import rt_hip

    for k, v in request.param.items():
        monkeypatch.setenv(k, v)
    r = rt_hip.Renderer(0, variant=knob_variant())
    yield r
    r.close()


@pytest.mark.parametrize("name", ["complex_97x61_d4", "medium_1280x720_d10", "synth200_1920x1080_d4",
                                  "synth10k_384x216_d6", "simple_2x2_d10"])
def test_stack_modes_golden(stack_renderer, name):
    rgb, st, m = _render(stack_renderer, name)
    assert rgb == golden_rgb(name), diff_summary(rgb, golden_rgb(name))
    assert {"primary": st.rays_primary, "shadow": st.rays_shadow, "reflect": st.rays_reflect} == m["rays"]


@pytest.mark.parametrize("depth", [0, 1, 2, 7, 64])
def test_stack_modes_depth_edges(stack_renderer, depth):
    import orc
    import rt_hip

    W, H = 67, 45
    sc = rt_hip.Scene.load(scene_path("medium"))
    stack_renderer.upload(sc)
    rgb, st = stack_renderer.render(sc.camera(), W, H, depth)
    ref, counts, _ = orc.OracleScene(scene_path("medium")).render(W, H, depth, threads=4)
    assert bytes(rgb) == ref, diff_summary(bytes(rgb), ref)
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (counts["primary"], counts["shadow"],
                                                                   counts["reflect"])
    rows = rt_hip.rows_for_shard(H, 8, 1, 3)
    rgb2, _ = stack_renderer.render(sc.camera(), W, H, depth, rows=rows)
    got = np.frombuffer(bytes(rgb2), np.uint8).reshape(-1, W, 3)
    want = np.frombuffer(ref, np.uint8).reshape(H, W, 3)
    for k in range(rows.count):
        y = (k // 8) * 8 * 3 + 8 + k % 8
        if y < H:
            assert np.array_equal(got[k], want[y])


@pytest.mark.parametrize("walk", [{}, {"RT_HIP_DEFER": "1"}, {"RT_HIP_BVH4": "0"}, {"RT_HIP_BVH_ORDERED": "0"}],
                         ids=["ordered4", "ordered4-defer", "ordered2", "stackless"])
@pytest.mark.parametrize("seed,count", [(101, 700), (102, 1100), (103, 1600)])
def test_large_scenes_global_memory_paths(monkeypatch, walk, seed, count):
    """Scenes read through L2 with the BVH fallback: the ordered 4-wide walk
    (default), the ordered two-child walk (RT_HIP_BVH4=0) and the stackless
    preorder walk (RT_HIP_BVH_ORDERED=0) against the oracle; above 1024 spheres
    every group walks the tree (384-cell shadow grids, 1-sphere leaves) and the
    deferred rays go through render_deferred (the uniform grid's closest hits)."""
    import orc
    import rt_hip

    for k, v in walk.items():
        monkeypatch.setenv(k, v)
    r = rt_hip.Renderer(0, variant=knob_variant())
    try:
        text = _random_scene(seed, count)
        W, H, D = 96, 64, 5
        sc = rt_hip.Scene.parse(text)
        r.upload(sc)
        ref, counts, _ = orc.OracleScene(text=text).render(W, H, D, threads=8)
        rgb, st = r.render(sc.camera(), W, H, D)
        assert bytes(rgb) == ref, diff_summary(bytes(rgb), ref)
        assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (counts["primary"], counts["shadow"],
                                                                       counts["reflect"])
    finally:
        r.close()


def _mirror_cloud(seed: int, n: int, frac: bool = False) -> str:
    """A camera inside a cloud of mirrors: nearly every pixel reflects at least
    twice, so the level-2 rays outnumber the deferred queue's room."""
    import random

    rng = random.Random(seed)
    lines = []
    for _ in range(n):
        lines.append("sphere %.6f %.6f %.6f %.6f %.3f %.3f %.3f %.2f 0.5 %s" % (
            rng.uniform(-14, 14), rng.uniform(-14, 14), rng.uniform(-14, 14), rng.uniform(0.6, 2.2),
            rng.random(), rng.random(), rng.random(), rng.choice([0.8, 0.9, 1.0]),
            _shininess(rng, True) if frac else "%d" % rng.choice([5, 20, 60])))
    lines.append("light 0 30 0 1 1 1 1")
    lines.append("light 20 -10 25 0.6 0.5 0.4 1")
    lines.append("ambient 0.1 0.1 0.1")
    lines.append("camera 0.3 0.2 0.1 5 1 -7 80")
    return "\n".join(lines) + "\n"


@pytest.mark.parametrize("n", [400, 1300], ids=["render_deferred", "render_deferred_walk"])
def test_deferred_queue_overflow_vs_oracle(n):
    """More level-2 rays than the deferred queue holds (room: 1/8 of the
    launch's pixels): the rays that find their shard segment full continue in
    the merged megakernel. Checked: the level-2 ray count exceeds the room; the
    image and ray counts equal a render without deferral (RT_HIP_DEFER=0); every
    31st row equals the oracle's.  n = 1300 takes the walk kernel
    (render_deferred_walk), n = 400 render_deferred.  These one-frame renders
    defer with RT_HIP_DEFER=1 (one-frame launches do not by default)."""
    import os

    import orc
    import rt_hip

    W, H, D = 512, 384, 6
    text = _mirror_cloud(7, n)
    sc = rt_hip.Scene.parse(text)
    old1 = os.environ.get("RT_HIP_DEFER")
    os.environ["RT_HIP_DEFER"] = "1"
    try:
        r = rt_hip.Renderer(0, variant=knob_variant())
    finally:
        if old1 is None:
            del os.environ["RT_HIP_DEFER"]
        else:
            os.environ["RT_HIP_DEFER"] = old1
    try:
        r.upload(sc)
        _, st2 = r.render(sc.camera(), W, H, 2)
        _, st3 = r.render(sc.camera(), W, H, 3)
        assert st3.rays_reflect - st2.rays_reflect > W * H // 8
        rgb, st = r.render(sc.camera(), W, H, D)
    finally:
        r.close()
    old = os.environ.get("RT_HIP_DEFER")
    os.environ["RT_HIP_DEFER"] = "0"
    try:
        r0 = rt_hip.Renderer(0, variant=knob_variant())
    finally:
        if old is None:
            del os.environ["RT_HIP_DEFER"]
        else:
            os.environ["RT_HIP_DEFER"] = old
    try:
        r0.upload(sc)
        rgb0, st0 = r0.render(sc.camera(), W, H, D)
    finally:
        r0.close()
    assert bytes(rgb) == bytes(rgb0), diff_summary(bytes(rgb), bytes(rgb0))
    assert (st.rays_primary, st.rays_shadow, st.rays_reflect) == (st0.rays_primary, st0.rays_shadow,
                                                                   st0.rays_reflect)
    full = np.frombuffer(bytes(rgb), np.uint8).reshape(H, W, 3)
    ref = orc.OracleScene(text=text)
    for y in range(0, H, 31):
        row, _, _ = ref.render(W, H, D, band=1, first=y, stride=1, count=1, threads=8)
        assert full[y].tobytes() == row, f"row {y}"


def test_cfg5_synth10k_4k_sampled_oracle_rows(gpu_renderer):
    """BASELINE cfg 5 at its full size (synth10k 3840x2160 d6: the uniform-grid
    closest hits, 768-cell shadow grids, the deferred kernel): every 64th row
    (rows 32, 96, ..., 2144) equals the oracle's."""
    import orc
    import rt_hip

    W, H, D = 3840, 2160, 6
    sc = rt_hip.Scene.load(scene_path("synth10k"))
    gpu_renderer.upload(sc)
    full, _ = gpu_renderer.render(sc.camera(), W, H, D)
    full = np.frombuffer(bytes(full), np.uint8).reshape(H, W, 3)
    ref = orc.OracleScene(scene_path("synth10k"))
    first, step = 32, 64
    count = (H - first + step - 1) // step
    rgb, _, _ = ref.render(W, H, D, band=1, first=first, stride=step, count=count, threads=16)
    want = np.frombuffer(rgb, np.uint8).reshape(count, W, 3)
    for i in range(count):
        y = first + i * step
        assert full[y].tobytes() == want[i].tobytes(), f"row {y}: {diff_summary(full[y].tobytes(), want[i].tobytes())}"
