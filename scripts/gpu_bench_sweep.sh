#!/bin/bash
# bench.py once per argument set (one per line of $SWEEP, default: frames per
# launch 16/24/32 at the default and at the driver's 20/5 step counts); prints
# value and kernel ms per frame.  Each run is time-limited; stops at a failure.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$ROOT"; mkdir -p gpurun_out/sweep
SWEEP="${SWEEP:-"--frames-per-launch 16
--frames-per-launch 24
--frames-per-launch 32
--steps 20 --warmup 5 --frames-per-launch 16
--steps 20 --warmup 5 --frames-per-launch 32"}"
i=0
while IFS= read -r args; do
  [ -z "$args" ] && continue
  out="gpurun_out/sweep/run$i"
  # leading VAR=value words of a line are environment settings for that run
  envs=(); rest=()
  for w in $args; do if [ ${#rest[@]} -eq 0 ] && [[ "$w" == *=* ]]; then envs+=("$w"); else rest+=("$w"); fi; done
  timeout -k 10 300 env "${envs[@]}" python bench.py --no-cpu-baseline "${rest[@]}" ${BENCH_ARGS} > "$out.json" 2> "$out.err" || { echo "rc=$? for $args"; tail -5 "$out.err"; exit 1; }
  python -c "
import json; d=json.load(open('$out.json')); a=d.get('also',{}).get('complex_1920x1080_d4',{})
print('%-55s %9.1f Mrays/s k=%.4f ms/frame launches=%s | complex %9.1f' % ('$args', d['value'], d['roofline']['kernel_ms_per_frame'], d['config']['launch_frames'], a.get('mrays_per_s',0)))"
  i=$((i+1))
done <<< "$SWEEP"
