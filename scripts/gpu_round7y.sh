# The other workloads' bench lines on the final tree (PMC-matched, profiles/r7x).
set -o pipefail
mkdir -p gpurun_out/r7y
export TMPDIR=/tmp
for w in complex_3840x2160_d4 synth10k_3840x2160_d6 complex_1920x1080_d4; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-also --workload $w > gpurun_out/r7y/bench_$w.json 2> gpurun_out/r7y/bench_$w.err || { tail -5 gpurun_out/r7y/bench_$w.err; exit 2; }
  python -c "
import json;d=json.loads(open('gpurun_out/r7y/bench_$w.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$w', d['value'], d['ms_per_step'], r['kernel_ms_per_frame'], r['frac'], r['lane_weighted'] and r['lane_weighted']['frac'], r['traffic'], d['config'].get('frame_equals_golden'), json.dumps(d.get('single_frame',{}).get('kernel_ms')))"
done
