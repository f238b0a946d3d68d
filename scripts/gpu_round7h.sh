set -o pipefail
mkdir -p gpurun_out/r7h
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread -rs > gpurun_out/r7h/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r7h/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r7h/pytest_gpu.log
grep "fuzz\[" gpurun_out/r7h/pytest_gpu.log || true
cd cs420-ray-tracer_amd && for i in 1 2 3; do ( time -p timeout -k 10 60 ./ray_serial --width 1920 --height 1080 --depth 4 scenes/complex.txt ) 2>&1 | tail -4; done; cd ..
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r7h/bench_20_5.json 2> gpurun_out/r7h/bench_20_5.err || exit 2
python -c "import json;d=json.loads(open('gpurun_out/r7h/bench_20_5.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step']);print(json.dumps(d['e2e']))"
