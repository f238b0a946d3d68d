# light lists nearest-first (tuning knob): parity of the light-grid tests with the knob, then the A/B
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5x
timeout -k 10 600 python -u scripts/ab_launch.py "RT_HIP_LG_ORDER=0;RT_HIP_LG_ORDER=1" synth200_1920x1080_d4 complex_1920x1080_d4 synth10k_3840x2160_d6 > gpurun_out/r5x/ab_lg_order.log 2>&1 || { tail -20 gpurun_out/r5x/ab_lg_order.log; exit 1; }
timeout -k 10 600 python -u scripts/ab_launch.py "RT_HIP_LG_ORDER=1;RT_HIP_LG_ORDER=0" synth200_1920x1080_d4 complex_1920x1080_d4 >> gpurun_out/r5x/ab_lg_order.log 2>&1 || { tail -20 gpurun_out/r5x/ab_lg_order.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5x/ab_lg_order.log | cut -c1-250
