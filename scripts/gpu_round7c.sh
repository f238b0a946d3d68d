set -o pipefail
mkdir -p gpurun_out/r7c
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_light_grid.py -m gpu -x -q -k "lazily or sphere_grid_scenes" --timeout 120 --timeout-method thread > gpurun_out/r7c/pytest_sg.log 2>&1 || { tail -30 gpurun_out/r7c/pytest_sg.log; exit 1; }
tail -2 gpurun_out/r7c/pytest_sg.log
timeout -k 10 120 python scripts/e2e_probe.py complex 6 > gpurun_out/r7c/e2e_probe.log 2>&1 || { cat gpurun_out/r7c/e2e_probe.log; exit 3; }
cat gpurun_out/r7c/e2e_probe.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r7c/bench_20_5.json 2> gpurun_out/r7c/bench_20_5.err || exit 2
python -c "import json;d=json.loads(open('gpurun_out/r7c/bench_20_5.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step']);print(json.dumps(d['e2e']));print(json.dumps(d['single_frame']))"
