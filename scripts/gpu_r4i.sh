#!/bin/bash
# Round-4: the warmup floor A/B -- the driver's --steps 20 --warmup 5 line with
# 0 / 50 ms of back-to-back warmup launches after the host-side builds,
# alternating, 3 reps each; then the default line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4i
for rep in 1 2 3; do
  for ws in 0 0.05; do
    BENCH_WARM_BUSY_S=$ws timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-also --no-extras > gpurun_out/r4i/b_${ws}_$rep.json 2> gpurun_out/r4i/b_${ws}_$rep.err || { echo "bench $ws failed"; tail -3 gpurun_out/r4i/b_${ws}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4i/b_${ws}_$rep.json')); print('warm_busy $ws rep $rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_frame'], d['config']['frame_equals_golden'], d['config']['warmup_frames_rendered'])"
  done
done
timeout -k 10 300 python bench.py > gpurun_out/r4i/bench_default.json 2> gpurun_out/r4i/bench_default.err || { echo default-failed; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4i/bench_default.json')); print('default', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'], d['moving_camera']['mrays_per_s'])"
timeout -k 10 400 python scripts/ab_launch.py "default;RT_HIP_CAM_GRID_N=256;RT_HIP_CAM_GRID_N=128;RT_HIP_CAM_GRID_N=64;RT_HIP_CAM_GRID=0" synth200_1920x1080_d4 complex_1920x1080_d4 > gpurun_out/r4i/ab_camgrid_n.log 2>&1 || { echo ab-camgrid-failed; exit 1; }
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_bench_dist.py > gpurun_out/r4i/pytest_bench_dist.log 2>&1 || { echo pytest-failed; exit 1; }
echo all-ok
