# device light grids + sphere grids (point_grids): parity suites, bench (e2e upload), synth10k upload
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5e
timeout -k 10 900 python -u -m pytest tests/test_light_grid.py tests/test_gpu_parity.py tests/test_behind_grid.py tests/test_gpu_check.py tests/test_gpu_frames.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5e/pytest.log 2>&1 || { tail -30 gpurun_out/r5e/pytest.log; exit 1; }
tail -2 gpurun_out/r5e/pytest.log
timeout -k 10 300 python bench.py > gpurun_out/r5e/bench.json 2> gpurun_out/r5e/bench.err || { tail -20 gpurun_out/r5e/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r5e/bench.json'));print(d['value'], d['e2e'])"
timeout -k 10 300 python bench.py --workload synth10k_3840x2160_d6 --steps 16 --warmup 8 --no-also --no-cpu-baseline > gpurun_out/r5e/bench_synth10k.json 2> gpurun_out/r5e/bench_synth10k.err || { tail -20 gpurun_out/r5e/bench_synth10k.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r5e/bench_synth10k.json'));print(d['value'], d['e2e'])"
