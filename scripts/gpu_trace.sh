#!/bin/bash
# Kernel-trace stats only (one bench run under rocprofv3), for pipeline breakdowns.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${TAG:-tr}"
W="${WORKLOAD:-synth200_1920x1080_d4}"
OUT="$ROOT/gpurun_out/trace_${TAG}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-also --workload "$W" --steps 20 --warmup 3 ${BENCH_ARGS} > "$OUT/bench.log" 2>&1
rc=$?
echo "rc=$rc"
f=$(find "$OUT" -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    print('%-70s n=%6s avg=%9.1f us tot=%8.2f ms %5.1f%%' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6, float(r['Percentage'])))
"
exit $rc
