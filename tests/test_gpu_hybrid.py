"""ray_hybrid (the hybrid CPU+GPU tile scheduler, SURVEY 8(f) row 4;
src/main_hybrid.cpp:321-830) on the GPU: argv grammar, stdout lines, the
tile split (estimate_tile_complexity, main_hybrid.cpp:323-347, against the
oracle's restatement), and the image -- every mode must write ray_serial's
image of the same size byte for byte (the golden fixtures rendered by the
reference's own trace_ray at the hybrid's 1080x720, depth 3)."""
import hashlib
import os
import re
import subprocess

import pytest

from conftest import PKG, golden_rgb, manifest, scene_path

pytestmark = pytest.mark.gpu


def run(tmp_path, *args, rc=0):
    r = subprocess.run([os.path.join(PKG, "ray_hybrid"), *args], cwd=tmp_path, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == rc, r.stdout + r.stderr
    return r.stdout


def p3_sha(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def split(scene, W, H, tile, thr):
    import orc

    t = orc.hybrid_tiles(orc.OracleScene(scene_path(scene)), W, H, tile, thr)
    return len(t), sum(1 for x in t if x[5])


@pytest.mark.parametrize("scene", ["simple", "medium", "complex"])
def test_default_mode_is_the_serial_image(tmp_path, scene):
    out = run(tmp_path, scene_path(scene))
    lines = out.splitlines()
    assert lines[0].startswith("Using GPU: ")
    assert "Tile size: 64x64" in lines
    assert f"Loading scene from: {scene_path(scene)}" in lines
    assert "Hybrid Rendering..." in lines
    n, ncpu = split(scene, 1080, 720, 64, 7)
    assert f"Created {n} tiles of size 64x64" in lines
    assert f"Distribution: {ncpu} tiles to CPU, {n - ncpu} tiles to GPU" in lines
    assert re.search(r"^Hybrid rendering time: [0-9.e+-]+ seconds$", out, re.M)
    assert lines[-1] == "Image written to output_hybrid.ppm"
    assert p3_sha(tmp_path / "output_hybrid.ppm") == manifest()[f"{scene}_1080x720_d3"]["sha256_p3"]


def test_pipeline_mode_uses_64_tiles_and_threshold_9(tmp_path):
    out = run(tmp_path, "-p", "-t", "32", "-o", "hyb.ppm", scene_path("complex"))
    n, ncpu = split("complex", 1080, 720, 64, 9)
    assert "Tile size: 32x32" in out and "Hybrid Pipeline Rendering..." in out
    assert f"Created {n} tiles of size 64x64" in out  # main_hybrid.cpp:790 passes no tile size
    assert f"Distribution: {ncpu} tiles to CPU, {n - ncpu} tiles to GPU" in out
    assert p3_sha(tmp_path / "hyb.ppm") == manifest()["complex_1080x720_d3"]["sha256_p3"]


@pytest.mark.parametrize("args", [["-t", "100"], ["--cpu-threshold", "-1", "-t", "128"],
                                  ["--cpu-threshold", "1000000"], ["--dynamic"], ["--dynamic", "--threads", "1"],
                                  ["--streams", "1", "-t", "37"]])
def test_every_split_gives_the_same_image(tmp_path, args):
    out = run(tmp_path, *args, scene_path("medium"))
    if "--cpu-threshold" in args and "-1" in args:
        assert re.search(r"Distribution: (\d+) tiles to CPU, 0 tiles to GPU", out)
    if "1000000" in args:
        assert re.search(r"Distribution: 0 tiles to CPU, \d+ tiles to GPU", out)
    assert p3_sha(tmp_path / "output_hybrid.ppm") == manifest()["medium_1080x720_d3"]["sha256_p3"]


def test_ragged_tiles_other_size(tmp_path):
    run(tmp_path, "--width", "97", "--height", "61", "--depth", "4", "-t", "16", "--cpu-threshold", "10",
        scene_path("complex"))
    data = open(tmp_path / "output_hybrid.ppm", "rb").read().split()
    assert data[:4] == [b"P3", b"97", b"61", b"255"]
    assert bytes(int(v) for v in data[4:]) == golden_rgb("complex_97x61_d4")


def test_missing_scene_fails_like_the_reference(tmp_path):
    r = subprocess.run([os.path.join(PKG, "ray_hybrid"), "no/such/scene.txt"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "Could not open scene file" in r.stderr
