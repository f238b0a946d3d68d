# the driver's N = 1 sequence on the final tree: smoke, bench at 20/5 and at the defaults
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6q
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6q/smoke.log 2>&1 || { tail -5 gpurun_out/r6q/smoke.log; exit 1; }
tail -1 gpurun_out/r6q/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6q/bench_20_5.json 2> gpurun_out/r6q/bench_20_5.err || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r6q/bench_default.json 2> gpurun_out/r6q/bench_default.err || exit 1
python - <<'PY'
import json
for f in ("bench_20_5", "bench_default"):
    d = json.load(open("gpurun_out/r6q/%s.json" % f))
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], r.get("flops_source"), r.get("pmc_matches_kernel_src"), r.get("frac"), r.get("valu_busy"), d["config"].get("frame_equals_golden", d["config"].get("golden_check")))
PY
