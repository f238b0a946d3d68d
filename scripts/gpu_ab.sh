#!/bin/bash
# Quick A/B: parity tests + bench with culling and brute force.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG="${TAG:-ab}"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
for variant in "" "--brute-force"; do
  timeout -k 10 600 python bench.py --no-cpu-baseline $variant ${BENCH_ARGS} > gpurun_out/bench_${TAG}$variant.json 2> gpurun_out/bench_${TAG}$variant.err; rc=$?
  echo "bench $variant rc=$rc"; python -c "
import json,sys; d=json.load(open('gpurun_out/bench_${TAG}$variant.json'))
print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'], d['roofline']['frac'], d['also'])"
  [ $rc -eq 0 ] || exit $rc
done
