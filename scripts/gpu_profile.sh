#!/bin/bash
# Round profile on one GPU: the default bench line, a rocprofv3 kernel trace of
# the same command, and the PMC passes (scripts/pmc_r2_passes.txt, one
# rocprofv3 run per pass) for each workload in $WORKLOADS.  Output under
# gpurun_out/prof_$TAG/ (then scripts/collect_round.sh).  Each GPU step has its own time limit; the script stops
# at the first failing step.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${TAG:-r2}"
OUT="$ROOT/gpurun_out/prof_$TAG"
WORKLOADS="${WORKLOADS:-synth200_1920x1080_d4 complex_1920x1080_d4 complex_3840x2160_d4 synth10k_3840x2160_d6}"
mkdir -p "$OUT"
# the kernel sources these runs measure (make_pmc_json.py records it with the PMC)
python3 -c "import sys; sys.path.insert(0, '$ROOT'); import bench; print(bench.kernel_source_sha())" > "$OUT/kernel_src_sha.txt"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 python3 "$ROOT/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -5 "$OUT/bench.err"; exit 1; }
echo "bench: $(head -c 300 "$OUT/bench.json")"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline --no-also --no-extras > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || { echo "trace failed"; tail -5 "$OUT/trace_bench.err"; exit 1; }
echo "trace ok"
# PMC passes: make_pmc_json.py folds the multi-frame launches only (32
# frames each at --steps 32 --warmup 16), so the product library runs as is
for w in $WORKLOADS; do
  i=0; mkdir -p "$OUT/pmc_$w"
  while IFS= read -r counters; do
    [ -z "$counters" ] && continue
    timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d "$OUT/pmc_$w/p$i" -o run -- \
      python3 "$ROOT/bench.py" --no-cpu-baseline --no-also --no-extras --workload "$w" --steps 32 --warmup 16 \
      > "$OUT/pmc_$w/p$i.log" 2>&1 || { echo "pmc $w pass $i failed"; tail -5 "$OUT/pmc_$w/p$i.log"; exit 1; }
    i=$((i+1))
  done < "$ROOT/scripts/pmc_r2_passes.txt"
  echo "pmc $w: $i passes"
done
