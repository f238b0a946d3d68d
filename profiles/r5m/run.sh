# one-frame launch shapes with a two-tile region: heavy classes single / in pairs / merged
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5m
timeout -k 10 900 python -u scripts/ab_launch.py "default;RT_HIP_SINGLE_CLASS=2+RT_HIP_PAIR_CLASS=1;RT_HIP_SINGLE_CLASS=3+RT_HIP_PAIR_CLASS=1;RT_HIP_SINGLE_CLASS=3+RT_HIP_PAIR_CLASS=2;RT_HIP_SINGLE_CLASS=1+RT_HIP_PAIR_CLASS=0" synth200_1920x1080_d4 complex_1920x1080_d4 > gpurun_out/r5m/ab_pairs.log 2>&1 || { tail -20 gpurun_out/r5m/ab_pairs.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5m/ab_pairs.log
