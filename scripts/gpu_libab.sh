#!/bin/bash
# A/B of library builds on one box: for each LIBS entry (a path under
# build_variants/, or "cur" = the in-tree librt_hip.so) run bench.py REPS
# times, alternating, on WORKLOAD (+ the complex "also" line).  Optional
# parity suite first (SKIP_TESTS=1 to skip).  Each GPU step is time-limited.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG="${TAG:-ab}"; REPS="${REPS:-3}"; W="${WORKLOAD:-synth200_1920x1080_d4}"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq 1 "$REPS"); do
  for spec in ${LIBS:-cur}; do
    # an entry may carry knobs: lib@K=V@K2=V2 (set for that entry's run only)
    lib="${spec%%@*}"; knobs=""; [ "$spec" != "$lib" ] && knobs="${spec#*@}"
    if [ "$lib" = cur ]; then unset RT_HIP_LIB; else export RT_HIP_LIB="$ROOT/$lib"; fi
    out="gpurun_out/${TAG}_$(basename "$lib" .so)$(echo "$knobs" | tr '@=' '__')_$rep"
    timeout -k 10 300 env $(echo "$knobs" | tr '@' ' ') python bench.py --no-cpu-baseline --workload "$W" --steps 64 ${BENCH_ARGS} > "$out.json" 2> "$out.err"; rc=$?
    [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 "$out.err"; exit $rc; }
    python -c "
import json; d=json.load(open('$out.json')); a=d['also'].get('complex_1920x1080_d4',{})
print('%-40s %s %9.1f Mrays/s k=%.4f ms/frame | complex %9.1f k=%.4f' % ('$spec', '$W'[:12], d['value'], d['roofline']['kernel_ms_per_frame'], a.get('mrays_per_s',0), a.get('kernel_ms_per_frame',0)))"
  done
done
