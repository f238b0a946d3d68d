#!/bin/bash
# The driver's step counts against the default: bench.py --steps 20 --warmup 5
# and the default 64/16, alternating REPS times (synth200, no extras), then a
# rocprofv3 kernel trace of the synth10k bench line.  Output in gpurun_out/.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
for rep in $(seq 1 "${REPS:-2}"); do
  for sw in "20 5" "64 16"; do
    set -- $sw
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps "$1" --warmup "$2" \
      > "gpurun_out/steps_$1_$2_$rep.json" 2> "gpurun_out/steps_$1_$2_$rep.err" || { echo "bench $sw failed"; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/steps_$1_$2_$rep.json'))
print('steps %s warmup %s: %.1f Mrays/s  %.4f ms/step  kernel %.4f ms/frame  launches %s' % ($1, $2, d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_frame'], d['config']['launch_frames']))"
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/trace10k" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline --no-also --no-extras --workload synth10k_3840x2160_d6 \
  > gpurun_out/trace10k.json 2> gpurun_out/trace10k.err || { echo "trace failed"; exit 1; }
echo "trace ok"
