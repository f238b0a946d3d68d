#!/bin/bash
# Round-4 batch: multi-frame parity with the single-tile tail, the tail A/B
# (tuning build, per-frame kernel time of 32/20/8-frame launches) and the
# driver's --steps 20 --warmup 5 line against build_variants/base.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4g
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_frames.py tests/test_gpu_bench_dist.py tests/test_behind_grid.py > gpurun_out/r4g/pytest.log 2>&1 || { echo pytest-fail; tail -5 gpurun_out/r4g/pytest.log; exit 1; }
tail -1 gpurun_out/r4g/pytest.log
timeout -k 10 500 python scripts/ab_launch.py "default;RT_HIP_TAIL=0" synth200_1920x1080_d4 complex_1920x1080_d4 synth10k_3840x2160_d6 > gpurun_out/r4g/ab_tail.log 2>&1 || { echo ab-launch-fail; exit 1; }
SKIP_TESTS=1 TAG=r4g/ab LIBS="build_variants/librt_hip_base.so cur" REPS=3 BENCH_ARGS="--no-extras --steps 20 --warmup 5" bash scripts/gpu_libab.sh > gpurun_out/r4g/ab_20_5.log 2>&1 || { echo ab-fail; exit 1; }
echo all-ok
