# bench line with the source-matched PMC, and the CLI tests (P3 writer bytes)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5j
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5j/bench_20_5.json 2> gpurun_out/r5j/bench.err || { tail -20 gpurun_out/r5j/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r5j/bench_20_5.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['frac'], r['flops_source'], r['valu_busy'], r['traffic'], d['e2e'])"
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_hybrid.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5j/pytest.log 2>&1 || { tail -30 gpurun_out/r5j/pytest.log; exit 1; }
tail -2 gpurun_out/r5j/pytest.log
