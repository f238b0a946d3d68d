# compiler scheduling strategies (same sources): library A/B, alternating
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6d
for rep in 1 2; do
  for lib in build_variants/librt_hip_r5y.so build_variants/librt_hip_memclause.so build_variants/librt_hip_trackers.so build_variants/librt_hip_both.so; do
    echo "== $lib rep $rep" >> gpurun_out/r6d/ab_lib.log
    RT_HIP_LIB="$GRAFT_REPO_ROOT/$lib" timeout -k 10 300 python -u scripts/ab_launch.py "default;RT_HIP_WIDE=3" synth200_1920x1080_d4 complex_1920x1080_d4 synth10k_3840x2160_d6 >> gpurun_out/r6d/ab_lib.log 2>&1 || { tail -20 gpurun_out/r6d/ab_lib.log; exit 1; }
  done
done
