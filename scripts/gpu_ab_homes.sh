# A/B of stack-home layouts (round 6): parity of each variant on the goldens
# and the bench launch shapes, PMC WRITE_SIZE per kernel, then bench timing
# alternating.  Variants under cs420-ray-tracer_amd/variants/exp/.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$ROOT"
OUT=gpurun_out/r7f; mkdir -p $OUT
export TMPDIR=/tmp
for v in ${VARIANTS:-lifo compact lifocompact}; do
  export RT_HIP_LIB=$ROOT/cs420-ray-tracer_amd/variants/exp/librt_hip_$v.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py -m gpu -x -q -k "golden or bench_launch_shape or deferred" --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { echo "parity $v failed"; tail -20 $OUT/pytest_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $OUT/pytest_$v.log)"
done
unset RT_HIP_LIB
for v in cur ${VARIANTS:-lifo compact lifocompact}; do
  if [ $v = cur ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$ROOT/cs420-ray-tracer_amd/variants/exp/librt_hip_$v.so; fi
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_$v -o run -- python3 bench.py --no-cpu-baseline --no-also --no-extras --workload synth200_1920x1080_d4 --steps 32 --warmup 16 > $OUT/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $OUT/pmc_$v.log; exit 1; }
done
for rep in 1 2; do
  for v in cur ${VARIANTS:-lifo compact lifocompact}; do
    if [ $v = cur ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$ROOT/cs420-ray-tracer_amd/variants/exp/librt_hip_$v.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 64 --warmup 16 > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err || exit 2
    python -c "
import json; d=json.loads(open('$OUT/bench_${v}_$rep.json').read().strip().splitlines()[-1]); a=d['also'].get('complex_1920x1080_d4',{})
print('%-12s %9.1f Mrays/s k=%.4f ms/frame | complex k=%.4f' % ('$v', d['value'], d['roofline']['kernel_ms_per_frame'], a.get('kernel_ms_per_frame',0)))"
  done
done
