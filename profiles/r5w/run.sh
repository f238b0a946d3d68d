# randomised parity sweeps on the final kernels: product library, and the tuning build with every launch's camera grid forced
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5w
timeout -k 10 400 python -u scripts/gpu_fuzz.py 330 5101 > gpurun_out/r5w/fuzz_default.log 2>&1 || { tail -20 gpurun_out/r5w/fuzz_default.log; exit 1; }
tail -2 gpurun_out/r5w/fuzz_default.log
FUZZ_VARIANT=tuning RT_HIP_CAM_GRID=2 timeout -k 10 400 python -u scripts/gpu_fuzz.py 330 5102 > gpurun_out/r5w/fuzz_camgrid2.log 2>&1 || { tail -20 gpurun_out/r5w/fuzz_camgrid2.log; exit 1; }
tail -2 gpurun_out/r5w/fuzz_camgrid2.log
