# Historical record (profiles/r7t): the A/B of the cooperative backward walk,
# commit d3980a4, reverted after it; variants/exp/ held the previous library.
# The wave-cooperative backward walk (kFastGrid kernels): parity on the scenes
# above 1,024 spheres (goldens, tangent scenes, fuzz), then cfg 5 and synth200
# against the previous library, alternating.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$ROOT"; OUT=gpurun_out/r7t; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_behind_grid.py tests/test_gpu_fuzz.py tests/test_gpu_frames.py tests/test_gpu_check.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
  for v in prev cur; do
    if [ $v = cur ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$ROOT/cs420-ray-tracer_amd/variants/exp/librt_hip_$v.so; fi
    for w in synth10k_3840x2160_d6 synth200_1920x1080_d4; do
      timeout -k 10 300 python bench.py --no-cpu-baseline --no-also --no-extras --workload $w > $OUT/b_${v}_${w}_$rep.json 2> $OUT/b_${v}_${w}_$rep.err || exit 2
      python -c "
import json;d=json.loads(open('$OUT/b_${v}_${w}_$rep.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$v', '$w', d['value'], r['kernel_ms_per_frame'])"
    done
  done
done
