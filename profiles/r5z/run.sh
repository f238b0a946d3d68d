# light-grid resolution re-swept with nearest-first lists (tuning build)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5z
timeout -k 10 600 python -u scripts/ab_launch.py "default;RT_HIP_SHADOW_GRID_N=384;RT_HIP_SHADOW_GRID_N=512;RT_HIP_SHADOW_GRID_N=1024" synth10k_3840x2160_d6 > gpurun_out/r5z/ab_lg_n.log 2>&1 || { tail -20 gpurun_out/r5z/ab_lg_n.log; exit 1; }
timeout -k 10 600 python -u scripts/ab_launch.py "default;RT_HIP_SHADOW_GRID_N=96;RT_HIP_SHADOW_GRID_N=192;RT_HIP_SHADOW_GRID_N=256" synth200_1920x1080_d4 complex_1920x1080_d4 >> gpurun_out/r5z/ab_lg_n.log 2>&1 || { tail -20 gpurun_out/r5z/ab_lg_n.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5z/ab_lg_n.log | cut -c1-60,130-260
