#!/bin/bash
# Tuning A/B on one box: each variant = (env assignments) run as separate bench processes.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG="${TAG:-var}"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
i=0
while IFS= read -r v; do
  [ -z "$v" ] && continue
  for rep in 1 2; do
    env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 64 ${BENCH_ARGS} > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err; rc=$?
    [ $rc -eq 0 ] || { echo "variant [$v] rc=$rc"; tail -5 gpurun_out/${TAG}_$i.err; exit $rc; }
    python -c "
import json; d=json.load(open('gpurun_out/${TAG}_$i.json')); a=d['also'].get('complex_1920x1080_d4',{})
print('%-60s synth200 %8.1f Mrays/s  k=%.4f ms/frame  complex %8.1f  k=%.4f' % ('$v', d['value'], d['roofline']['kernel_ms_per_frame'], a.get('mrays_per_s',0), a.get('kernel_ms_per_frame',0)))"
  done
  i=$((i+1))
done < "${VARIANTS:-scripts/variants.txt}"
