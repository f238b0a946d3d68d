"""Hybrid CPU+GPU tile scheduler (ray_hybrid, SURVEY 8(f) row 4;
src/main_hybrid.cpp:321-830), host side: the CPU tile worker (csrc/rt_cpu.cpp)
and the tile cost model against the oracle, without a GPU.

Parity: the worker's image must equal the oracle's -- and the golden fixtures
rendered by the reference's own trace_ray -- byte for byte; the tile costs
must equal oracle/rt_oracle.c's restatement of estimate_tile_complexity
(main_hybrid.cpp:323-347).  The reference's hybrid driver itself cannot be
built here (it needs CUDA), so the cost model is pinned only by that
restatement ("parity unpinned" for the split counts; they decide where a tile
is rendered, never its pixels)."""
import os
import subprocess
import sys

import pytest

from conftest import golden_rgb, manifest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "cs420-ray-tracer_amd")
CSRC = os.path.join(PKG, "csrc")
sys.path.insert(0, os.path.join(REPO, "oracle"))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = tmp_path_factory.mktemp("hyb") / "cpu_tiles_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-I", CSRC,
                    "-I", os.path.join(REPO, "include"), "-o", str(exe),
                    os.path.join(REPO, "tests", "native", "cpu_tiles_check.cpp"), os.path.join(CSRC, "rt_cpu.cpp"),
                    "-L", PKG, "-lrt_hip", "-Wl,-rpath," + PKG], check=True)
    return str(exe)


def run_checker(exe, tmp_path, scene, W, H, D, tile):
    rgb, costs = tmp_path / "rgb.bin", tmp_path / "costs.txt"
    subprocess.run([exe, os.path.join(PKG, "scenes", scene + ".txt"), str(W), str(H), str(D), str(tile),
                    str(rgb), str(costs)], check=True, timeout=600)
    return rgb.read_bytes(), [int(v) for v in costs.read_text().split()]


@pytest.mark.parametrize("name,tile", [("simple_1080x720_d3", 64), ("complex_97x61_d4", 16), ("simple_2x2_d10", 64),
                                       ("medium_1080x720_d3", 100)])
def test_cpu_tiles_equal_golden(checker, tmp_path, name, tile):
    import orc

    m = manifest()[name]
    rgb, costs = run_checker(checker, tmp_path, m["scene"], m["width"], m["height"], m["depth"], tile)
    assert rgb == golden_rgb(name)
    sc = orc.OracleScene(os.path.join(PKG, "scenes", m["scene"] + ".txt"))
    want = [c for (_, _, _, _, c, _) in orc.hybrid_tiles(sc, m["width"], m["height"], tile, 7)]
    assert costs == want


def test_hybrid_cli_help_needs_no_gpu():
    exe = os.path.join(PKG, "ray_hybrid")
    out = subprocess.run([exe, "--help"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0
    assert "--pipeline, -p" in out.stdout and "--tile-size, -t SIZE" in out.stdout


def test_ray_hybrid_not_in_library():
    """The CPU tile worker is linked into ray_hybrid only: librt_hip.so has no
    CPU render path (no rtc:: symbols)."""
    out = subprocess.run(["nm", "-DC", os.path.join(PKG, "librt_hip.so")], capture_output=True, text=True, check=True)
    assert "rtc::" not in out.stdout and "CpuTracer" not in out.stdout
