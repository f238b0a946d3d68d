#!/bin/bash
# One GPU session: smoke, the full parity suite, bench lines at the driver's
# and the default step counts, the rocprofv3 counter list.  Every GPU step has
# its own time limit; the script stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -4 "gpurun_out/$name.log"
  return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread &&
step bench_20_5 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline &&
step bench_64_16 300 python bench.py --steps 64 --warmup 16 --no-cpu-baseline &&
step counters 120 rocprofv3 -L
