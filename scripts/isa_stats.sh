#!/bin/bash
# Register / spill metadata of the render kernels for the working tree (or a
# git revision): bash scripts/isa_stats.sh [REV] [extra hipcc flags]
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
REV="${1:-WORKTREE}"; shift || true
TMP=$(mktemp -d)
if [ "$REV" = WORKTREE ]; then SRC="$ROOT/cs420-ray-tracer_amd/csrc"; INC="$ROOT/include"
else
  mkdir -p "$TMP/csrc" "$TMP/include"
  for f in $(git -C "$ROOT" ls-tree --name-only "$REV" cs420-ray-tracer_amd/csrc/); do git -C "$ROOT" show "$REV:$f" > "$TMP/csrc/$(basename "$f")"; done
  git -C "$ROOT" show "$REV:include/rt_hip.h" > "$TMP/include/rt_hip.h"
  SRC="$TMP/csrc"; INC="$TMP/include"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I"$INC" "$@" --cuda-device-only -S \
  -o "$TMP/k.s" "$SRC/rt_kernel.hip" 2>/dev/null
python3 - "$TMP/k.s" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
meta = txt[txt.rfind("amdhsa.kernels"):]
for blk in meta.split("  - .")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or "render" not in name.group(1): continue
    g = lambda k: (re.search(r"\.%s:\s+(\d+)" % k, blk) or [None, "?"])[1]
    print("%-60s vgpr %s spill %s | sgpr %s spill %s | lds %s" % (name.group(1)[:60], g("vgpr_count"), g("vgpr_spill_count"), g("sgpr_count"), g("sgpr_spill_count"), g("group_segment_fixed_size")))
PY
rm -rf "$TMP"
