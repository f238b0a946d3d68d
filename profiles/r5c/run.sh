# device sphere grids: parity suites, then the bench line (e2e upload)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5c
timeout -k 10 900 python -u -m pytest tests/test_light_grid.py tests/test_gpu_parity.py tests/test_behind_grid.py tests/test_gpu_check.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5c/pytest.log 2>&1 || { tail -30 gpurun_out/r5c/pytest.log; exit 1; }
tail -2 gpurun_out/r5c/pytest.log
timeout -k 10 300 python bench.py > gpurun_out/r5c/bench.json 2> gpurun_out/r5c/bench.err || { tail -20 gpurun_out/r5c/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r5c/bench.json'));print(d['value'], d['e2e'], d['config']['sphere_grids'])"
