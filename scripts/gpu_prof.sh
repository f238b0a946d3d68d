#!/bin/bash
# Profile pass: kernel trace + stats of the bench workload, then PMC passes
# (each counter group in its own run, --pmc only with kernel-trace output).
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${TAG:-r1}"
W="${WORKLOAD:-synth200_1920x1080_d4}"
OUT="$ROOT/gpurun_out/prof_${TAG}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-also --workload "$W" --steps 20 --warmup 3 ${BENCH_ARGS} > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -h '"value"' "$OUT/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); print(' value', d['value'], 'kernel_ms', d['roofline']['kernel_ms_mean'])"
  return $rc
}
run trace --kernel-trace --stats || exit $?
run pmc_fetch --pmc FETCH_SIZE || exit $?
run pmc_write --pmc WRITE_SIZE || exit $?
run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY || exit $?
run pmc_grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
ls -R "$OUT" | head -40
