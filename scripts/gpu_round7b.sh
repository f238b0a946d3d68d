set -o pipefail
mkdir -p gpurun_out/r7b
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 420 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r7b/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r7b/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r7b/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r7b/bench_20_5.json 2> gpurun_out/r7b/bench_20_5.err || exit 2
timeout -k 10 120 python scripts/e2e_probe.py complex 5 > gpurun_out/r7b/e2e_probe.log 2>&1 || exit 3
cat gpurun_out/r7b/e2e_probe.log
timeout -k 10 180 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --stats -d gpurun_out/r7b/e2e_prof -o e2e --output-format csv -- python3 scripts/e2e_probe.py complex 3 > gpurun_out/r7b/e2e_prof.log 2>&1 || exit 4
echo done
