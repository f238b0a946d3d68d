#!/bin/bash
# Round evidence in one GPU call: parity tests, the bench line (with CPU
# baselines), a rocprofv3 kernel trace of the default workload, and PMC passes
# for the synth200 / complex / synth10k workloads.  Output: gpurun_out/round_$TAG/
# (copy into profiles/ with scripts/collect_round.sh).
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${TAG:-r1}"
OUT="$ROOT/gpurun_out/round_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -m pytest tests -m gpu -q > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-also --steps 64 --warmup 16 > "$OUT/trace_bench.json" 2> "$OUT/trace.err" || { tail -5 "$OUT/trace.err"; exit 1; }
echo "trace ok"
for w in synth200_1920x1080_d4 complex_1920x1080_d4 synth10k_3840x2160_d6; do
  PASSES="$ROOT/scripts/pmc_traffic_passes.txt" TAG="round_$TAG/pmc_$w" WORKLOAD=$w bash "$ROOT/scripts/gpu_pmc.sh" || exit 1
done
