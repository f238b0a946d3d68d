# shadow-line bound (off_free), shared-reciprocal division variant, one-frame shape re-sweep, one-frame timeline
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5u
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5u/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5u/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r5u/pytest_gpu.log
RT_HIP_LIB="$GRAFT_REPO_ROOT/build_variants/librt_hip_fastdiv.so" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_divcheck.py -x -q --timeout 300 --timeout-method thread -k "golden or random or mirror or fractional or div" > gpurun_out/r5u/pytest_fastdiv.log 2>&1 || { tail -30 gpurun_out/r5u/pytest_fastdiv.log; exit 1; }
tail -2 gpurun_out/r5u/pytest_fastdiv.log
for rep in 1 2; do
  for lib in build_variants/librt_hip_r5x.so cs420-ray-tracer_amd/librt_hip.so build_variants/librt_hip_fastdiv.so; do
    echo "== $lib rep $rep" >> gpurun_out/r5u/ab_lib.log
    RT_HIP_LIB="$GRAFT_REPO_ROOT/$lib" timeout -k 10 300 python -u scripts/ab_launch.py "default;RT_HIP_WIDE=3" synth200_1920x1080_d4 complex_1920x1080_d4 synth10k_3840x2160_d6 >> gpurun_out/r5u/ab_lib.log 2>&1 || { tail -20 gpurun_out/r5u/ab_lib.log; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/r5u/ab_lib.log | tail -4
# one-frame launch shape re-swept with the wide light loop (tuning build)
timeout -k 10 300 python -u scripts/ab_launch.py "default;RT_HIP_SINGLE_CLASS=2;RT_HIP_SINGLE_CLASS=3;RT_HIP_SINGLE_CLASS=9;RT_HIP_TAIL_WAVES=6;RT_HIP_TAIL_WAVES=24" synth200_1920x1080_d4 complex_1920x1080_d4 > gpurun_out/r5u/ab_one_frame.log 2>&1 || { tail -20 gpurun_out/r5u/ab_one_frame.log; exit 1; }
# one-frame timeline (stamps build: per-wave start / end)
RT_HIP_LIB="$GRAFT_REPO_ROOT/build_variants/librt_hip_stamps.so" RT_HIP_STAMPS_FILE="$GRAFT_REPO_ROOT/gpurun_out/r5u/tl1.bin" timeout -k 10 120 python -u scripts/timeline.py synth200 1920 1080 4 > gpurun_out/r5u/tl1.log 2>&1 || { tail -20 gpurun_out/r5u/tl1.log; exit 1; }
tail -3 gpurun_out/r5u/tl1.log
