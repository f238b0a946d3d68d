# max-memory-clause scheduling in the product build: the GPU suite, then the round profile on these sources and flags
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6e/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r6e/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6e/pytest_gpu.log
TAG=r6e bash scripts/gpu_profile.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6e/bench_20_5.json 2> gpurun_out/r6e/bench_20_5.err || exit 1
