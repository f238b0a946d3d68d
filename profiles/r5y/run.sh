# nearest-first light lists by default: the GPU suite, then the round profile on these sources
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5y
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5y/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5y/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r5y/pytest_gpu.log
TAG=r5y bash scripts/gpu_profile.sh || exit 1
