"""The drop-in CLI (ray_serial / ray_openmp / ray_hip) on the GPU, as the
reference's makefile:48-96 and scripts/test.sh:207-224 drive ray_serial /
ray_openmp: output file names, stdout lines, and the P3 bytes (SHA-256 of the
reference's own output)."""
import hashlib
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import PKG, golden_rgb, manifest, scene_path

pytestmark = pytest.mark.gpu


def run(tmp_path, exe, *args):
    r = subprocess.run([os.path.join(PKG, exe), *args], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def sha(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def test_ray_serial_default_size_is_the_reference_bytes(tmp_path):
    out = run(tmp_path, "ray_serial", scene_path("simple"))
    assert "Loaded scene: 5 spheres, 2 lights" in out
    assert "Serial time:" in out and "seconds" in out
    assert sha(tmp_path / "output_serial.ppm") == manifest()["simple_1280x720_d10"]["sha256_p3"]
    assert os.path.getsize(tmp_path / "output_serial.ppm") >= 1000  # scripts/test.sh:207-224


def test_ray_openmp_writes_both_passes(tmp_path):
    out = run(tmp_path, "ray_openmp", scene_path("medium"))
    assert "Serial time:" in out and "OpenMP time:" in out
    want = manifest()["medium_1280x720_d10"]["sha256_p3"]
    assert sha(tmp_path / "output_serial.ppm") == want
    assert sha(tmp_path / "output_openmp.ppm") == want


def test_ray_openmp_flag_renders_only_the_openmp_pass(tmp_path):
    out = run(tmp_path, "ray_openmp", "--openmp", scene_path("complex"))
    assert "OpenMP time:" in out and "Serial time:" not in out
    assert not (tmp_path / "output_serial.ppm").exists()
    assert sha(tmp_path / "output_openmp.ppm") == manifest()["complex_1280x720_d10"]["sha256_p3"]


def test_ray_hip_sizes_and_p6(tmp_path):
    name = "complex_1920x1080_d4"
    out = run(tmp_path, "ray_hip", "--width", "1920", "--height", "1080", "--depth", "4", "--p6",
              scene_path("complex"))
    assert "GPU rendering time:" in out
    data = open(tmp_path / "output_gpu.ppm", "rb").read()
    head = b"P6\n1920 1080\n255\n"
    assert data.startswith(head) and data[len(head):] == golden_rgb(name)


def test_ray_hip_antialias(tmp_path):
    import orc

    run(tmp_path, "ray_hip", "-a", "--width", "96", "--height", "54", "--depth", "4", "--p6", "--out", "aa.ppm",
        scene_path("complex"))
    data = open(tmp_path / "aa.ppm", "rb").read()
    ref, _, _ = orc.OracleScene(scene_path("complex")).render_aa(96, 54, 4, samples=4, threads=4)
    assert data.endswith(ref) and len(data) == len(b"P6\n96 54\n255\n") + len(ref)


def test_ray_hip_missing_scene_fails_like_the_reference(tmp_path):
    r = subprocess.run([os.path.join(PKG, "ray_hip"), "no_such_scene.txt"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "Could not open scene file" in r.stderr


def test_ray_hip_gather_path_one_gpu(tmp_path):
    """The --gpus G code path (ncclCommInitAll, ncclGather to device 0,
    unpermute) rehearsed with G = 1."""
    run(tmp_path, "ray_hip", "--gpus", "1", "--force-gather", "--width", "1920", "--height", "1080", "--depth", "4",
        "--p6", scene_path("complex"))
    data = open(tmp_path / "output_gpu.ppm", "rb").read()
    assert data.endswith(golden_rgb("complex_1920x1080_d4"))


def test_ray_hip_multi_gpu_gather(tmp_path):
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs (the row gather over RCCL); covered by tests/test_multirank.py on CPU")
    run(tmp_path, "ray_hip", "--gpus", "2", "--width", "1920", "--height", "1080", "--depth", "4", "--p6",
        scene_path("complex"))
    data = open(tmp_path / "output_gpu.ppm", "rb").read()
    assert data.endswith(golden_rgb("complex_1920x1080_d4"))
