"""CPU-only: the product's host side (librt_hip.so loads without a GPU): every
header symbol is exported, the scene parser matches the reference loader's
grammar (via the oracle's restatement), the camera basis is bit-identical, the
P3 writer is byte-identical to write_ppm, and the synthetic scenes are
reproducible."""
import hashlib
import os
import re
import subprocess

import pytest

import orc
import rt_hip
from conftest import GOLDEN, PKG, REPO, golden_rgb, manifest, scene_path

HEADER = os.path.join(REPO, "include", "rt_hip.h")


def header_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(rt_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    names = header_functions()
    assert len(names) >= 20
    out = subprocess.check_output(["nm", "-D", "--defined-only", rt_hip.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    assert set(names) == set(rt_hip.SIGNATURES), "ctypes binding out of sync with rt_hip.h"
    lib = rt_hip.lib()
    for n in names:
        getattr(lib, n)
    assert lib.rt_abi_version() == rt_hip.ABI_VERSION == 12


def test_error_strings():
    for code in range(8):
        assert rt_hip.status_string(code)
    assert rt_hip.status_string(0) == "ok"


@pytest.mark.parametrize("name", ["simple", "medium", "complex", "synth200", "synth10k"])
def test_parser_matches_oracle_on_scene_files(name):
    s = rt_hip.Scene.load(scene_path(name))
    o = orc.OracleScene(scene_path(name))
    assert (s.num_spheres, s.num_lights) == (o.s.num_spheres, o.s.num_lights)
    for i in range(s.num_spheres):
        a, b = s.sphere(i), o.s.spheres[i]
        assert a["center"] == (b.center.x, b.center.y, b.center.z)
        assert a["radius"] == b.radius and a["reflectivity"] == b.reflectivity and a["shininess"] == b.shininess
        assert a["color"] == (b.color.x, b.color.y, b.color.z)
    for i in range(s.num_lights):
        a, b = s.light(i), o.s.lights[i]
        assert a["position"] == (b.position.x, b.position.y, b.position.z)
        assert a["color"] == (b.color.x, b.color.y, b.color.z)
    assert tuple(s.raw.ambient) == (o.s.ambient.x, o.s.ambient.y, o.s.ambient.z)


def test_scene_sizes_are_the_real_ones():
    # the headers say 200 / 50, the files hold 154 / 44
    assert rt_hip.Scene.load(scene_path("complex")).num_spheres == 154
    assert rt_hip.Scene.load(scene_path("medium")).num_spheres == 44
    assert rt_hip.Scene.load(scene_path("synth200")).num_spheres == 200


QUIRKS = """
# comment
   # indented comment
\t  sphere 1 2 3 0.5 1 0 0 0.2 0.9 30 extra tokens ignored
sphere 1 2 3 oops 1 0 0 0.2 0.9 30
sphere 1 2 3
light 1 2 3 1 1 1
light 4 5 6 0.5 0.5 0.5 1.0
ambient 0.1 0.2
ambient 0.3 0.3 0.3
ambient 0.4 0.5 0.6
camera 0 0 0 0 0 -1
camera 1 2 3 4 5 6 45
teapot 1 2 3
sphere 1e1 -2.5e-1 +3. .5 1 1 1 0 0 1
sphere 1x 2 3 4 1 1 1 0 0 1
sphere 1.5.5 2 3 4 1 1 1 0 0 1
sphere 1e999 2 3 4 1 1 1 0 0 1
sphere 1e-999 2 3 4 1 1 1 0 0 1
"""


@pytest.mark.parametrize("text", [QUIRKS, "", "\n\n", "camera 1 1 1 0 0 0 90", "sphere 0 0 -5 1 1 1 1 0 0 1\r\n"
                                  "light 0 5 0 1 1 1 1\r\n"])
def test_parser_quirks_match_oracle(text):
    s = rt_hip.Scene.parse(text)
    o = orc.OracleScene(text=text)
    assert (s.num_spheres, s.num_lights, s.warnings) == (o.s.num_spheres, o.s.num_lights, o.s.warnings)
    for i in range(s.num_spheres):
        assert s.sphere(i)["center"] == (o.s.spheres[i].center.x, o.s.spheres[i].center.y, o.s.spheres[i].center.z)
        assert s.sphere(i)["radius"] == o.s.spheres[i].radius
    assert tuple(s.raw.ambient) == (o.s.ambient.x, o.s.ambient.y, o.s.ambient.z)
    assert tuple(s.raw.cam_position) == (o.s.cam_position.x, o.s.cam_position.y, o.s.cam_position.z)
    assert s.raw.cam_fov == o.s.cam_fov and s.raw.has_camera == o.s.has_camera


def test_parser_quirk_details():
    s = rt_hip.Scene.parse(QUIRKS)
    # kept: the first, the exponent one, "1.5.5" (istream reads 1.5 then .5) and
    # 1e-999 (underflow is accepted); "1x", "oops", the short one and 1e999 are skipped
    assert s.num_spheres == 4
    assert s.sphere(2)["center"] == (1.5, 0.5, 2.0) and s.sphere(2)["radius"] == 3.0
    assert s.sphere(3)["center"][0] == 0.0
    assert s.num_lights == 1
    assert tuple(s.raw.ambient) == (0.4, 0.5, 0.6)  # last valid one wins
    assert tuple(s.raw.cam_position) == (1, 2, 3) and s.raw.cam_fov == 45
    assert s.sphere(1)["center"] == (10.0, -0.25, 3.0) and s.sphere(1)["radius"] == 0.5


def test_missing_scene_is_an_io_error():
    with pytest.raises(rt_hip.RtError) as e:
        rt_hip.Scene.load("/nonexistent/scene.txt")
    assert e.value.status == 6


def test_default_camera_when_absent():
    s = rt_hip.Scene.parse("sphere 0 0 -5 1 1 1 1 0 0 1")
    c = s.camera()
    assert tuple(c.position) == (0, 0, 0) and tuple(c.forward) == (0, 0, -1)  # scene.h:22


@pytest.mark.parametrize("name", ["simple", "medium", "complex", "synth200"])
def test_camera_basis_bit_identical(name):
    c = rt_hip.Scene.load(scene_path(name)).camera()
    o = orc.OracleScene(scene_path(name)).camera()
    for f in ("position", "forward", "right", "up"):
        v = getattr(o, f)
        assert tuple(getattr(c, f)) == (v.x, v.y, v.z), f
    assert c.scale == o.scale


@pytest.mark.parametrize("name", ["complex_97x61_d4", "simple_800x600_d10", "complex_1920x1080_d4"])
def test_p3_writer_byte_identical_to_reference(tmp_path, name):
    m = manifest()[name]
    p = tmp_path / "out.ppm"
    rt_hip.write_ppm(str(p), golden_rgb(name), m["width"], m["height"])
    assert hashlib.sha256(p.read_bytes()).hexdigest() == m["sha256_p3"]


@pytest.mark.parametrize("name", ["complex_97x61_d4", "complex_1920x1080_d4"])
def test_p3_writer_through_a_pipe(tmp_path, name):
    """A file that cannot be sized and mapped (a FIFO): the writer formats its
    pixel ranges into buffers and writes them in order -- the same bytes."""
    import threading

    m = manifest()[name]
    fifo = tmp_path / "out.fifo"
    os.mkfifo(fifo)
    got = []
    reader = threading.Thread(target=lambda: got.append(open(fifo, "rb").read()))
    reader.start()
    assert rt_hip.write_ppm(str(fifo), golden_rgb(name), m["width"], m["height"]) is None
    reader.join(60)
    assert hashlib.sha256(got[0]).hexdigest() == m["sha256_p3"]


def test_p3_writer_edge_sizes(tmp_path):
    """Empty and one-pixel images, and ranges whose last pixel is short
    ("0 0 0\n") at every chunk boundary of the parallel path."""
    import numpy as np

    for W, H in ((0, 0), (1, 1), (3, 0), (1000, 300)):
        rgb = (np.arange(W * H * 3) % 7 == 0).astype(np.uint8) * 200 if W * H else np.zeros(0, np.uint8)
        p = tmp_path / ("e%dx%d.ppm" % (W, H))
        rt_hip.write_ppm(str(p), rgb.tobytes(), W, H)
        want = "P3\n%d %d\n255\n" % (W, H) + "".join(
            "%d %d %d\n" % tuple(rgb[3 * i:3 * i + 3]) for i in range(W * H))
        assert p.read_bytes() == want.encode(), (W, H)


def test_p6_writer(tmp_path):
    m = manifest()["complex_97x61_d4"]
    p = tmp_path / "out.ppm"
    rgb = golden_rgb("complex_97x61_d4")
    rt_hip.write_ppm(str(p), rgb, m["width"], m["height"], binary=True)
    assert p.read_bytes() == b"P6\n97 61\n255\n" + rgb


@pytest.mark.parametrize("name", ["synth200", "synth10k"])
def test_synthetic_scenes_reproducible(name):
    import synth

    assert synth.generate(name) == open(scene_path(name)).read()


def test_rows_for_shard_covers_every_row_once():
    for H in (1, 7, 61, 1080, 2160):
        for band in (1, 8, 16):
            for G in (1, 2, 3, 8):
                seen = []
                for r in range(G):
                    rows = rt_hip.rows_for_shard(H, band, r, G)
                    for k in range(rows.count):
                        y = (k // band) * band * G + r * band + k % band
                        if y < H:
                            seen.append(y)
                assert sorted(seen) == list(range(H))
                # rt_rows_for_shard: one row count for every rank (the gather's equal shards)
                assert len({rt_hip.rows_for_shard(H, band, r, G).count for r in range(G)}) == 1


def test_rows_for_shard_rejects_bad_layouts():
    for args in ((1080, 0, 0, 1), (1080, 8, 2, 2), (1080, 8, -1, 2), (1080, 8, 0, 0), (-1, 8, 0, 1)):
        with pytest.raises(rt_hip.RtError):
            rt_hip.rows_for_shard(*args)


def test_cli_usage_exits_cleanly():
    r = subprocess.run([os.path.join(PKG, "ray_hip"), "--help"], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


def test_compat_interface_exported_with_reference_layouts():
    """include/rt_hip_compat.h: launch_gpu_kernel / upload_lights_and_ambience are
    exported by librt_hip.so, and the structs have the reference's layouts
    (float3 12 B, GPUMaterial 20 B, GPUSphere 36 B, GPULight 28 B, GPUCamera 88 B,
    include/gpu_shared.h:84-171)."""
    import ctypes as C

    text = open(os.path.join(REPO, "include", "rt_hip_compat.h")).read()
    names = sorted(set(re.findall(r"^\s*(?:void|int)\s+(\w+)\s*\(", text, re.M)))
    assert names == sorted(rt_hip.COMPAT_SIGNATURES), names
    out = subprocess.check_output(["nm", "-D", "--defined-only", rt_hip.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert set(names) <= exported
    sizes = {rt_hip.rt_float3: 12, rt_hip.rt_gpu_material: 20, rt_hip.rt_gpu_sphere: 36, rt_hip.rt_gpu_light: 28,
             rt_hip.rt_gpu_camera: 88}
    for t, n in sizes.items():
        assert C.sizeof(t) == n, (t.__name__, C.sizeof(t))
    assert rt_hip.lib().rt_compat_status() == 0
