# more randomised parity sweeps: the lane-per-ray light loop (tuning build), and a new seed at both sizes
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6r
FUZZ_VARIANT=tuning RT_HIP_WIDE=0 FUZZ_NEAR_LIGHTS=1 timeout -k 10 400 python -u scripts/gpu_fuzz.py 280 9301 > gpurun_out/r6r/fuzz_wide0_9301.log 2>&1 || { tail -3 gpurun_out/r6r/fuzz_wide0_9301.log; exit 1; }
tail -1 gpurun_out/r6r/fuzz_wide0_9301.log
FUZZ_NEAR_LIGHTS=1 timeout -k 10 400 python -u scripts/gpu_fuzz.py 280 9302 > gpurun_out/r6r/fuzz_near_9302.log 2>&1 || { tail -3 gpurun_out/r6r/fuzz_near_9302.log; exit 1; }
tail -1 gpurun_out/r6r/fuzz_near_9302.log
FUZZ_LARGE=1 timeout -k 10 400 python -u scripts/gpu_fuzz.py 280 9303 > gpurun_out/r6r/fuzz_large_9303.log 2>&1 || { tail -3 gpurun_out/r6r/fuzz_large_9303.log; exit 1; }
tail -1 gpurun_out/r6r/fuzz_large_9303.log
