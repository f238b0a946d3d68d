#!/bin/bash
# Per-shard kernel-time probe (scripts/shard_probe.py) under several env variants.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
WL="${WL:-synth200_1920x1080_d4}"
while IFS= read -r v; do
  [ -z "$v" ] && continue
  out=$(env $v timeout -k 10 120 python scripts/shard_probe.py $WL ${FRAMES:-15} 2>gpurun_out/shv.err) || { echo "[$v] failed"; tail -5 gpurun_out/shv.err; exit 1; }
  echo "$out" | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('%-50s G1 %.4f  G2 %.4f  G4 %.4f  G8 %.4f ms  eff8 %.3f' % ('$v', d['G1']['max_ms'], d['G2']['max_ms'], d['G4']['max_ms'], d['G8']['max_ms'], d['G8']['kernel_eff']))"
done < "${VARIANTS:-scripts/variants.txt}"
