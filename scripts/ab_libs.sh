#!/bin/bash
# Launch-shape A/B of library builds on one box: for each LIBS entry (a path
# under build_variants/, or "cur" = the in-tree librt_hip.so), alternating REPS
# times, scripts/ab_launch.py with the default knobs on WORKLOADS.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
for rep in $(seq 1 "${REPS:-2}"); do
  for lib in ${LIBS:-cur}; do
    if [ "$lib" = cur ]; then unset RT_HIP_LIB; else export RT_HIP_LIB="$ROOT/$lib"; fi
    echo "== $lib rep $rep"
    timeout -k 10 300 python -u scripts/ab_launch.py RT_HIP_SINGLE_CLASS=default ${WORKLOADS} 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
