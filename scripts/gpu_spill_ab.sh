#!/bin/bash
# Parity tests, then bench lines for three workloads and the FETCH/WRITE PMC passes.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG="${TAG:-spill}"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
for w in synth200_1920x1080_d4 complex_1920x1080_d4 synth10k_3840x2160_d6; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-also --workload $w > gpurun_out/bench_${TAG}_$w.json 2> gpurun_out/bench_${TAG}_$w.err; rc=$?
  echo "bench $w rc=$rc"; cat gpurun_out/bench_${TAG}_$w.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_mean'))"
  [ $rc -eq 0 ] || exit $rc
done
TAG=${TAG}_fw PASSES="$ROOT/scripts/pmc_fw.txt" bash "$ROOT/scripts/gpu_pmc.sh" || exit 1
python3 "$ROOT/scripts/pmc_summary.py" "$ROOT/gpurun_out/${TAG}_fw" 2>&1 | tail -20
