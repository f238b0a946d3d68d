# randomised parity sweeps at 1,024+ tiles per frame (the heavy-first tile order), with near lights
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6o
FUZZ_LARGE=1 FUZZ_NEAR_LIGHTS=1 timeout -k 10 500 python -u scripts/gpu_fuzz.py 420 9101 > gpurun_out/r6o/fuzz_large_9101.log 2>&1 || { tail -3 gpurun_out/r6o/fuzz_large_9101.log; exit 1; }
tail -1 gpurun_out/r6o/fuzz_large_9101.log
FUZZ_LARGE=1 FUZZ_VARIANT=tuning RT_HIP_CAM_GRID=2 timeout -k 10 500 python -u scripts/gpu_fuzz.py 420 9102 > gpurun_out/r6o/fuzz_large_camgrid2_9102.log 2>&1 || { tail -3 gpurun_out/r6o/fuzz_large_camgrid2_9102.log; exit 1; }
tail -1 gpurun_out/r6o/fuzz_large_camgrid2_9102.log
