cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5b
timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_check.py tests/test_light_grid.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5b/pytest.log 2>&1 || { tail -30 gpurun_out/r5b/pytest.log; exit 1; }
tail -3 gpurun_out/r5b/pytest.log
RT_HIP_CAM_GRID=2 timeout -k 10 330 python -u scripts/gpu_fuzz.py 300 11 > gpurun_out/r5b/fuzz_camgrid2.log 2>&1 || { tail -5 gpurun_out/r5b/fuzz_camgrid2.log; exit 1; }
tail -2 gpurun_out/r5b/fuzz_camgrid2.log
