# The driver's N = 1 sequence on the current tree: smoke, bench at 20/5 and at
# the defaults, each line PMC-matched (profiles/pmc_traffic.json).
set -o pipefail
mkdir -p gpurun_out/r7q
export TMPDIR=/tmp
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r7q/smoke.log 2>&1 || { cat gpurun_out/r7q/smoke.log; exit 1; }
tail -1 gpurun_out/r7q/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r7q/bench_20_5.json 2> gpurun_out/r7q/bench_20_5.err || exit 2
timeout -k 10 300 python bench.py > gpurun_out/r7q/bench_default.json 2> gpurun_out/r7q/bench_default.err || exit 3
for f in bench_20_5 bench_default; do python -c "
import json;d=json.loads(open('gpurun_out/r7q/$f.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$f', d['value'], d['ms_per_step'], r['frac'], r['lane_weighted'], r['traffic'], d['config']['frame_equals_golden'])"; done
