# one-frame launch shapes: single tiles vs merged class 0 with a single-tile tail, deferral, a camera grid per launch
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5g
timeout -k 10 900 python -u scripts/ab_launch.py "default;RT_HIP_SINGLE_CLASS=1;RT_HIP_SINGLE_CLASS=2;RT_HIP_SINGLE_CLASS=1+RT_HIP_DEFER=1;RT_HIP_CAM_GRID=2+RT_HIP_CAM_GRID_N=128;RT_HIP_CAM_GRID=2+RT_HIP_CAM_GRID_N=64;RT_HIP_CAM_GRID=2+RT_HIP_CAM_GRID_N=128+RT_HIP_SINGLE_CLASS=1" synth200_1920x1080_d4 complex_1920x1080_d4 > gpurun_out/r5g/ab_one_frame.log 2>&1 || { tail -20 gpurun_out/r5g/ab_one_frame.log; exit 1; }
cat gpurun_out/r5g/ab_one_frame.log
