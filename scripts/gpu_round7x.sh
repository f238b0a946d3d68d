# The final tree, as the driver runs it at round end on one GPU: smoke, the
# bench at 20/5 and at its defaults (each line PMC-matched against
# profiles/pmc_traffic.json), then the whole GPU suite and the drop-in CLI.
set -o pipefail
OUT=gpurun_out/r7x_drv
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_20_5.json 2> $OUT/bench_20_5.err || exit 2
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 3
for f in bench_20_5 bench_default; do python -c "
import json;d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$f', d['value'], d['ms_per_step'], r['frac'], r['lane_weighted'], r['traffic'], d['config']['frame_equals_golden'])"; done
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread -rs > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 4; }
tail -3 $OUT/pytest_gpu.log
cd cs420-ray-tracer_amd && for i in 1 2 3; do ( time -p timeout -k 10 60 ./ray_serial --width 1920 --height 1080 --depth 4 scenes/complex.txt ) 2>&1 | tail -4; done
