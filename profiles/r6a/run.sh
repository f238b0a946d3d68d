# one-frame launches with the device camera grid built per launch (tuning build), grid sizes
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6a
timeout -k 10 600 python -u scripts/ab_launch.py "default;RT_HIP_CAM_GRID=2;RT_HIP_CAM_GRID=2+RT_HIP_CAM_GRID_N=64;RT_HIP_CAM_GRID=2+RT_HIP_CAM_GRID_N=96;RT_HIP_CAM_GRID=2+RT_HIP_CAM_GRID_N=192" synth200_1920x1080_d4 complex_1920x1080_d4 > gpurun_out/r6a/ab_one_frame_grid.log 2>&1 || { tail -20 gpurun_out/r6a/ab_one_frame_grid.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6a/ab_one_frame_grid.log | cut -c1-140
