# deferral level / room re-swept on the final kernels (tuning build)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6g
timeout -k 10 600 python -u scripts/ab_launch.py "default;RT_HIP_DEFER_LEVEL=3;RT_HIP_DEFER_LEVEL=1;RT_HIP_DEFER_DIV=4" synth10k_3840x2160_d6 synth200_1920x1080_d4 > gpurun_out/r6g/ab_defer.log 2>&1 || { tail -20 gpurun_out/r6g/ab_defer.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6g/ab_defer.log | cut -c1-70,200-300
