# the wide light loop in passes (sparse and half-full waves): parity, then the A/B
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5o
timeout -k 10 600 python -u -m pytest tests/test_gpu_frames.py -x -v -k "wide" --timeout 300 --timeout-method thread > gpurun_out/r5o/pytest.log 2>&1 || { tail -30 gpurun_out/r5o/pytest.log; exit 1; }
tail -2 gpurun_out/r5o/pytest.log
timeout -k 10 600 python -u scripts/ab_launch.py "default;RT_HIP_WIDE=1;RT_HIP_WIDE=2" synth200_1920x1080_d4 complex_1920x1080_d4 synth10k_3840x2160_d6 > gpurun_out/r5o/ab_wide.log 2>&1 || { tail -20 gpurun_out/r5o/ab_wide.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5o/ab_wide.log
