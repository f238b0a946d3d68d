#!/bin/bash
# Round-4 batch: GPU suite, library A/B vs base (bench extras), and one-frame
# per-wave timelines (stamps build) of synth200 1080p and complex 4K.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r4m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest-fail; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
SKIP_TESTS=1 TAG=${TAG:-r4m}/ab LIBS="${LIBS:-build_variants/librt_hip_base.so cur}" REPS=${REPS:-3} BENCH_ARGS="--no-cpu-baseline --no-also" bash scripts/gpu_libab.sh > $O/ab.log 2>&1 || { echo ab-fail; tail -3 $O/ab.log; exit 1; }
tail -6 $O/ab.log
if [ -n "$TIMELINE" ]; then
  RT_HIP_LIB=$PWD/build_variants/librt_hip_stamps.so RT_HIP_STAMPS_FILE=/tmp/tl.bin timeout -k 10 120 python scripts/timeline_frames.py synth200 1920 1080 4 1 > $O/timeline_synth200_f1.log 2>&1 || { echo tl-fail; tail -3 $O/timeline_synth200_f1.log; exit 1; }
  RT_HIP_LIB=$PWD/build_variants/librt_hip_stamps.so RT_HIP_STAMPS_FILE=/tmp/tl.bin timeout -k 10 120 python scripts/timeline_frames.py complex 3840 2160 4 1 > $O/timeline_complex4k_f1.log 2>&1 || { echo tl-fail; tail -3 $O/timeline_complex4k_f1.log; exit 1; }
fi
echo all-ok
