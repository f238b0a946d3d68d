#!/bin/bash
# Round-end evidence on one GPU (after scripts/gpu_profile.sh + collect_round.sh
# put a PMC record matching these sources in profiles/pmc_traffic.json): the GPU
# suite, bench lines with the matched PMC (default, the driver's 20/5, cfg 5,
# cfg 4, complex), and the row-shard projection (scripts/shard_probe.py, 32
# frames per launch).  Output under gpurun_out/final_$TAG/; stops at the first
# failing step.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${TAG:-r3}"
OUT="$ROOT/gpurun_out/final_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -5 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python bench.py > "$OUT/bench_pmc_matched.json" 2> "$OUT/bench.err" || { echo "bench failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_20_5_pmc_matched.json" 2> "$OUT/bench_20_5.err" || { echo "bench 20/5 failed"; exit 1; }
for w in synth10k_3840x2160_d6 complex_3840x2160_d4; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-also --no-extras > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { echo "bench $w failed"; exit 1; }
done
for w in synth200_1920x1080_d4 complex_3840x2160_d4 synth10k_3840x2160_d6; do
  FPL=32 timeout -k 10 300 python scripts/shard_probe.py $w 64 > "$OUT/shard_$w.json" 2> "$OUT/shard_$w.err" || { echo "shard probe $w failed"; exit 1; }
done
echo "final ok"
