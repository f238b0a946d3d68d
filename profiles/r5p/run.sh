# wide light loop default on every fp64 launch; mode 3 adds it to the deferred kernel
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5p
timeout -k 10 600 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5p/pytest.log 2>&1 || { tail -30 gpurun_out/r5p/pytest.log; exit 1; }
tail -2 gpurun_out/r5p/pytest.log
timeout -k 10 600 python -u scripts/ab_launch.py "default;RT_HIP_WIDE=0;RT_HIP_WIDE=3" synth200_1920x1080_d4 complex_1920x1080_d4 synth10k_3840x2160_d6 > gpurun_out/r5p/ab_wide.log 2>&1 || { tail -20 gpurun_out/r5p/ab_wide.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5p/ab_wide.log
