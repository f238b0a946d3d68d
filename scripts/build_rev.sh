#!/bin/bash
# Build librt_hip.so from the kernel sources of git revision REV (default HEAD)
# into build_variants/librt_hip_NAME.so, for A/B runs (RT_HIP_LIB=...).
#   bash scripts/build_rev.sh REV NAME [extra hipcc defines]
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
REV="${1:-HEAD}"; NAME="${2:-base}"; shift 2 || true
TMP=$(mktemp -d)
mkdir -p "$TMP/csrc" "$TMP/include" "$ROOT/build_variants"
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" cs420-ray-tracer_amd/csrc/); do
  git -C "$ROOT" show "$REV:$f" > "$TMP/csrc/$(basename "$f")"
done
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" include/); do
  git -C "$ROOT" show "$REV:$f" > "$TMP/include/$(basename "$f")"
done
cd "$TMP/csrc"
SRCS=$(ls rt_kernel.hip rt_bvh.cpp rt_lightgrid.cpp rt_sched.cpp rt_host.cpp rt_compat.cpp 2>/dev/null || true)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -I../include "$@" -shared \
  -o "$ROOT/build_variants/librt_hip_$NAME.so" $SRCS
rm -rf "$TMP"
echo "built build_variants/librt_hip_$NAME.so from $REV"
