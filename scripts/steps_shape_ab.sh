cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --frames-per-launch 20" "--steps 40 --warmup 16" "--steps 32 --warmup 16" "--steps 64 --warmup 16"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-also $args > gpurun_out/s2.json 2> gpurun_out/s2.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/s2.json'))
print('%-48s %9.1f Mrays/s %.4f ms/step kernel %.4f launches %s' % ('$args', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_frame'], d['config']['launch_frames']))"
done
done
