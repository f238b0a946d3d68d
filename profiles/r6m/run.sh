# the round profile on the fixed sources, then the camera-grid-forced fuzz
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6m
TAG=r6m bash scripts/gpu_profile.sh || exit 1
FUZZ_VARIANT=tuning RT_HIP_CAM_GRID=2 timeout -k 10 400 python -u scripts/gpu_fuzz.py 300 7102 > gpurun_out/r6m/fuzz_camgrid2.log 2>&1 || { tail -3 gpurun_out/r6m/fuzz_camgrid2.log; exit 1; }
tail -1 gpurun_out/r6m/fuzz_camgrid2.log
