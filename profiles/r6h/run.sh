# randomised parity sweeps on the final build: product library, and the tuning build with every launch's camera grid forced
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6h
timeout -k 10 400 python -u scripts/gpu_fuzz.py 330 7101 > gpurun_out/r6h/fuzz_default.log 2>&1 || { tail -20 gpurun_out/r6h/fuzz_default.log; exit 1; }
tail -1 gpurun_out/r6h/fuzz_default.log
FUZZ_VARIANT=tuning RT_HIP_CAM_GRID=2 timeout -k 10 400 python -u scripts/gpu_fuzz.py 330 7102 > gpurun_out/r6h/fuzz_camgrid2.log 2>&1 || { tail -20 gpurun_out/r6h/fuzz_camgrid2.log; exit 1; }
tail -1 gpurun_out/r6h/fuzz_camgrid2.log
