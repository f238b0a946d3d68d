#!/bin/bash
# Copy a scripts/gpu_profile.sh result (gpurun_out/prof_$TAG) into
# profiles/$TAG and fold its PMC passes into profiles/pmc_traffic.json.
#   TAG=r2e bash scripts/collect_round.sh
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
TAG="${TAG:-r2}"
SRC="$ROOT/gpurun_out/prof_$TAG"
DST="$ROOT/profiles/$TAG"
mkdir -p "$DST"
cp "$SRC/bench.json" "$DST/"
[ -f "$SRC/kernel_src_sha.txt" ] && cp "$SRC/kernel_src_sha.txt" "$DST/"
cp "$SRC"/trace/run_kernel_stats.csv "$DST/kernel_stats.csv"
python3 "$ROOT/scripts/prof_summary.py" "$SRC/trace/run_kernel_trace.csv" --labels synth200 > "$DST/trace_summary.json"
cp "$SRC/trace_bench.json" "$DST/trace_bench.json"
for d in "$SRC"/pmc_*; do
  w=$(basename "$d"); w=${w#pmc_}
  mkdir -p "$DST/pmc/$w"
  for p in "$d"/p*/; do
    mkdir -p "$DST/pmc/$w/$(basename "$p")"
    cp "$p"/run_counter_collection.csv "$DST/pmc/$w/$(basename "$p")/"
  done
  python3 "$ROOT/scripts/make_pmc_json.py" "$w" "$DST/pmc/$w"
done
