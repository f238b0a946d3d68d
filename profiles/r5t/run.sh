# the normal formed once per hit (+ sqrt-free decisions): parity, then same-box library A/B (previous build vs current), alternating
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5t
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5t/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5t/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r5t/pytest_gpu.log
for rep in 1 2; do
  for lib in build_variants/librt_hip_r5w.so cs420-ray-tracer_amd/librt_hip.so; do
    echo "== $lib rep $rep" >> gpurun_out/r5t/ab_lib.log
    RT_HIP_LIB="$GRAFT_REPO_ROOT/$lib" timeout -k 10 300 python -u scripts/ab_launch.py "default;RT_HIP_WIDE=3" synth200_1920x1080_d4 complex_1920x1080_d4 synth10k_3840x2160_d6 >> gpurun_out/r5t/ab_lib.log 2>&1 || { tail -20 gpurun_out/r5t/ab_lib.log; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/r5t/ab_lib.log
