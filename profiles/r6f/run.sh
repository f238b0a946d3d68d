# render_deferred at 4 waves per SIMD (128 VGPRs), 48 or 64 workgroups per shard: library A/B
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6f
for rep in 1 2; do
  for lib in cs420-ray-tracer_amd/librt_hip.so build_variants/librt_hip_defer4.so build_variants/librt_hip_defer4w48.so; do
    echo "== $lib rep $rep" >> gpurun_out/r6f/ab_lib.log
    RT_HIP_LIB="$GRAFT_REPO_ROOT/$lib" timeout -k 10 300 python -u scripts/ab_launch.py "default;RT_HIP_WIDE=3" synth200_1920x1080_d4 synth10k_3840x2160_d6 >> gpurun_out/r6f/ab_lib.log 2>&1 || { tail -20 gpurun_out/r6f/ab_lib.log; exit 1; }
  done
done
