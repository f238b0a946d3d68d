#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over the bench workload.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${TAG:-pmc}"
W="${WORKLOAD:-synth200_1920x1080_d4}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
PASSES="${PASSES:-scripts/pmc_passes.txt}"
case "$PASSES" in /*) ;; *) PASSES="$ROOT/$PASSES";; esac
[ -f "$PASSES" ] || { echo "no pass file $PASSES"; exit 1; }
export TMPDIR=/tmp
cd /tmp
i=0
while IFS= read -r counters; do
  [ -z "$counters" ] && continue
  timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-also --workload "$W" --steps 32 --warmup 16 ${BENCH_ARGS} > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  i=$((i+1))
done < "$PASSES"
echo "pmc passes: $i"
