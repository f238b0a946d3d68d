#!/bin/bash
# Round-4 camera-grid build probe: a kernel trace of the bench (its single-frame
# and moving-camera extras build device grids), then library A/B vs base.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out/r4j
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r4j/trace" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-also > "$R/gpurun_out/r4j/trace.json" 2> "$R/gpurun_out/r4j/trace.err") || { echo trace-fail; tail -5 gpurun_out/r4j/trace.err; exit 1; }
echo trace-ok
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4j/pytest_gpu.log 2>&1 || { echo pytest-fail; tail -5 gpurun_out/r4j/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/r4j/pytest_gpu.log
fi
if [ -n "$KNOBS" ]; then
  timeout -k 10 400 python scripts/ab_launch.py "$KNOBS" synth200_1920x1080_d4 complex_1920x1080_d4 > gpurun_out/r4j/ab_knobs.log 2>&1 || { echo ab-knobs-failed; tail -5 gpurun_out/r4j/ab_knobs.log; exit 1; }
  grep same_image gpurun_out/r4j/ab_knobs.log
fi
SKIP_TESTS=1 TAG=r4j/ab LIBS="${LIBS:-build_variants/librt_hip_base.so cur}" REPS=${REPS:-2} BENCH_ARGS="--no-cpu-baseline --no-also" bash scripts/gpu_libab.sh > gpurun_out/r4j/ab.log 2>&1 || { echo ab-fail; exit 1; }
echo all-ok
