# randomised sweep on the bounds-checked build (every device index range-checked; a violation raises RT_ERR_CHECK)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6p
FUZZ_VARIANT=check FUZZ_NEAR_LIGHTS=1 timeout -k 10 400 python -u scripts/gpu_fuzz.py 300 9201 > gpurun_out/r6p/fuzz_check_9201.log 2>&1 || { tail -5 gpurun_out/r6p/fuzz_check_9201.log; exit 1; }
tail -1 gpurun_out/r6p/fuzz_check_9201.log
FUZZ_VARIANT=check FUZZ_LARGE=1 timeout -k 10 400 python -u scripts/gpu_fuzz.py 300 9202 > gpurun_out/r6p/fuzz_check_large_9202.log 2>&1 || { tail -5 gpurun_out/r6p/fuzz_check_large_9202.log; exit 1; }
tail -1 gpurun_out/r6p/fuzz_check_large_9202.log
