# cfg 5 diagnostic: the whole-line grid walk vs a forward-only walk (not exact:
# the ceiling of any speed-up of the backward part), alternating.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$ROOT"; mkdir -p gpurun_out/r7s; export TMPDIR=/tmp
for rep in 1 2; do
  for v in cur fwdonly; do
    if [ $v = cur ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$ROOT/cs420-ray-tracer_amd/variants/exp/librt_hip_$v.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-also --no-extras --workload synth10k_3840x2160_d6 > gpurun_out/r7s/b_${v}_$rep.json 2> gpurun_out/r7s/b_${v}_$rep.err || exit 2
    python -c "
import json;d=json.loads(open('gpurun_out/r7s/b_${v}_$rep.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$v', d['value'], r['kernel_ms_per_frame'])"
  done
done
