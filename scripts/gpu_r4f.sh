#!/bin/bash
# Round-4 batch: the GPU suite on the working tree, then library A/B with the
# bench's extras (single frame, moving camera) against build_variants/base.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4f/pytest_gpu.log 2>&1 || { echo pytest-fail; tail -5 gpurun_out/r4f/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4f/pytest_gpu.log
SKIP_TESTS=1 TAG=r4f/ab LIBS="${LIBS:-build_variants/librt_hip_base.so cur}" REPS=${REPS:-3} BENCH_ARGS="--no-cpu-baseline" bash scripts/gpu_libab.sh > gpurun_out/r4f/ab.log 2>&1 || { echo ab-fail; exit 1; }
echo all-ok
