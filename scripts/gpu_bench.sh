#!/bin/bash
# GPU session: parity tests, bench line, rocprofv3 kernel trace of the same bench.
# Each GPU step has its own time limit; stop at the first crash-like exit.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG="${TAG:-r1}"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_${TAG}.json; tail -5 gpurun_out/bench_${TAG}.err
[ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_PROF" ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_${TAG}" -o bench -- python3 "$ROOT/bench.py" --no-cpu-baseline ${BENCH_ARGS} > "$ROOT/gpurun_out/prof_${TAG}.log" 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -3 "$ROOT/gpurun_out/prof_${TAG}.log"
  find "$ROOT/gpurun_out/prof_${TAG}" -name "*stats*" | head
fi
