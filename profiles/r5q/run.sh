# the full GPU suite on the wide-by-default kernels
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5q
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5q/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r5q/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r5q/pytest_gpu.log
