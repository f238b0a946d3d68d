# more randomised parity sweeps on the final build: lights just outside spheres, new seeds, the camera grid forced
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6n
FUZZ_NEAR_LIGHTS=1 timeout -k 10 400 python -u scripts/gpu_fuzz.py 330 8101 > gpurun_out/r6n/fuzz_near_8101.log 2>&1 || { tail -3 gpurun_out/r6n/fuzz_near_8101.log; exit 1; }
tail -1 gpurun_out/r6n/fuzz_near_8101.log
timeout -k 10 400 python -u scripts/gpu_fuzz.py 330 8102 > gpurun_out/r6n/fuzz_8102.log 2>&1 || { tail -3 gpurun_out/r6n/fuzz_8102.log; exit 1; }
tail -1 gpurun_out/r6n/fuzz_8102.log
FUZZ_NEAR_LIGHTS=1 FUZZ_VARIANT=tuning RT_HIP_CAM_GRID=2 timeout -k 10 400 python -u scripts/gpu_fuzz.py 300 8103 > gpurun_out/r6n/fuzz_near_camgrid2_8103.log 2>&1 || { tail -3 gpurun_out/r6n/fuzz_near_camgrid2_8103.log; exit 1; }
tail -1 gpurun_out/r6n/fuzz_near_camgrid2_8103.log
