set -o pipefail
mkdir -p gpurun_out/r7e
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_cli.py tests/test_light_grid.py -m gpu -x -q -k "cli or lazily" --timeout 120 --timeout-method thread > gpurun_out/r7e/pytest.log 2>&1 || { tail -30 gpurun_out/r7e/pytest.log; exit 1; }
tail -2 gpurun_out/r7e/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r7e/bench_20_5.json 2> gpurun_out/r7e/bench_20_5.err || exit 2
python -c "import json;d=json.loads(open('gpurun_out/r7e/bench_20_5.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step']);print(json.dumps(d['e2e']))"
cd cs420-ray-tracer_amd && for i in 1 2 3; do ( time -p timeout -k 10 60 ./ray_serial --width 1920 --height 1080 --depth 4 scenes/complex.txt ) 2>&1 | tail -4; done
