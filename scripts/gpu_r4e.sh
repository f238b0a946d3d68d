#!/bin/bash
# Round-4 experiment batch: device sqrt check, library A/B (HEAD base / the
# sqrt core / + out-of-line exact test), stamps phases + one-frame timeline,
# launch-shape knobs (issue priority, one-tile classes) on the tuning build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4d gpurun_out/r4e
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_renorm.py > gpurun_out/r4e/pytest_renorm.log 2>&1 || { echo renorm-fail; exit 1; }
SKIP_TESTS=1 TAG=r4e/ab LIBS="build_variants/librt_hip_base.so cur build_variants/librt_hip_ni.so" REPS=2 BENCH_ARGS="--no-extras" bash scripts/gpu_libab.sh > gpurun_out/r4e/ab.log 2>&1 || { echo ab-fail; exit 1; }
timeout -k 10 400 python scripts/ab_launch.py "default;RT_HIP_PRIO=1;RT_HIP_PRIO=2;RT_HIP_SINGLE_CLASS=1;RT_HIP_SINGLE_CLASS=1+RT_HIP_PRIO=1" synth200_1920x1080_d4 complex_1920x1080_d4 > gpurun_out/r4e/ab_launch.log 2>&1 || { echo ab-launch-fail; exit 1; }
( export RT_HIP_LIB=build_variants/librt_hip_stamps.so RT_HIP_STAMPS=1
  timeout -k 10 120 python scripts/phase_stamps.py synth200 1920 1080 4 16 > gpurun_out/r4d/s200.log 2>&1 &&
  timeout -k 10 120 python scripts/phase_stamps.py synth200 1920 1080 4 1 > gpurun_out/r4d/s200_1.log 2>&1 &&
  timeout -k 10 200 python scripts/phase_stamps.py synth10k 3840 2160 6 4 > gpurun_out/r4d/s10k.log 2>&1 &&
  RT_HIP_STAMPS_FILE=/tmp/tl1.bin timeout -k 10 120 python scripts/timeline.py synth200 1920 1080 4 > gpurun_out/r4d/tl1.log 2>&1 &&
  python scripts/timeline.py --analyse /tmp/tl1.bin >> gpurun_out/r4d/tl1.log 2>&1 ) || { echo stamps-fail; exit 1; }
echo all-ok
