# the driver's round-end sequence on the final tree: smoke, the GPU suite, bench at 20/5 and at the defaults
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6b
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6b/smoke.log 2>&1 || { tail -20 gpurun_out/r6b/smoke.log; exit 1; }
tail -1 gpurun_out/r6b/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6b/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r6b/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6b/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6b/bench_20_5.json 2> gpurun_out/r6b/bench_20_5.err || { tail -5 gpurun_out/r6b/bench_20_5.err; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/r6b/bench_default.json 2> gpurun_out/r6b/bench_default.err || { tail -5 gpurun_out/r6b/bench_default.err; exit 1; }
python - <<'PY'
import json
for f in ("bench_20_5", "bench_default"):
    d = json.load(open("gpurun_out/r6b/%s.json" % f))
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], r.get("flops_source"), r.get("pmc_matches_kernel_src"), r.get("frac"), r.get("traffic"), r.get("valu_busy"))
PY
