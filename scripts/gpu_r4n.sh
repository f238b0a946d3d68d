#!/bin/bash
# Round-4 drain-mode batch: its GPU tests, the GPU suite, then library A/B
# (product vs the tuning build at RT_HIP_DRAIN=0/1/2) with the bench extras.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r4n}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_drain.py -x -v --timeout 120 --timeout-method thread > $O/pytest_drain.log 2>&1 || { echo drain-tests-fail; tail -15 $O/pytest_drain.log; exit 1; }
tail -1 $O/pytest_drain.log
if [ -z "$NOSUITE" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest-fail; tail -5 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
T=cs420-ray-tracer_amd/variants/librt_hip_tuning.so
SKIP_TESTS=1 TAG=${TAG:-r4n}/ab LIBS="${LIBS:-build_variants/librt_hip_base.so cur $T@RT_HIP_DRAIN=1 $T@RT_HIP_DRAIN=2}" REPS=${REPS:-2} BENCH_ARGS="--no-cpu-baseline ${BENCH_EXTRA}" bash scripts/gpu_libab.sh > $O/ab.log 2>&1 || { echo ab-fail; tail -3 $O/ab.log; exit 1; }
tail -8 $O/ab.log
echo all-ok
