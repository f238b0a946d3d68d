#!/bin/bash
# Kernel traces of the default bench line (static view, no extras) for each
# library in LIBS ("cur" = in-tree), to compare per-kernel durations.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
OUT="$R/gpurun_out/${TAG:-r4k}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in ${LIBS:-build_variants/librt_hip_base.so cur}; do
  if [ "$lib" = cur ]; then unset RT_HIP_LIB; name=cur; else export RT_HIP_LIB="$R/$lib"; name=$(basename "$lib" .so); fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$name" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-also --no-extras ${BENCH_ARGS} > "$OUT/$name.json" 2> "$OUT/$name.err") || { echo "trace $name failed"; tail -5 "$OUT/$name.err"; exit 1; }
  echo "$name: $(head -c 160 "$OUT/$name.json")"
done
echo all-ok
