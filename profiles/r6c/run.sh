# camera grid built beside one-frame launches (tuning knob), then the product library against the previous build
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6c
FUZZ_VARIANT=tuning RT_HIP_CAM_GRID_OVERLAP=1 timeout -k 10 200 python -u scripts/gpu_fuzz.py 120 6101 > gpurun_out/r6c/fuzz_overlap.log 2>&1 || { tail -20 gpurun_out/r6c/fuzz_overlap.log; exit 1; }
tail -1 gpurun_out/r6c/fuzz_overlap.log
timeout -k 10 600 python -u scripts/ab_launch.py "default;RT_HIP_CAM_GRID_OVERLAP=1;RT_HIP_CAM_GRID_OVERLAP=1+RT_HIP_CAM_GRID_N=96" synth200_1920x1080_d4 complex_1920x1080_d4 > gpurun_out/r6c/ab_overlap.log 2>&1 || { tail -20 gpurun_out/r6c/ab_overlap.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6c/ab_overlap.log | cut -c1-110
for rep in 1 2; do
  for lib in build_variants/librt_hip_r5y.so cs420-ray-tracer_amd/librt_hip.so; do
    echo "== $lib rep $rep" >> gpurun_out/r6c/ab_lib.log
    RT_HIP_LIB="$GRAFT_REPO_ROOT/$lib" timeout -k 10 300 python -u scripts/ab_launch.py "default;RT_HIP_WIDE=3" synth200_1920x1080_d4 synth10k_3840x2160_d6 >> gpurun_out/r6c/ab_lib.log 2>&1 || { tail -20 gpurun_out/r6c/ab_lib.log; exit 1; }
  done
done
