# stack homes + deferred-slot stacks: the GPU suite, then the bench lines (scratch, per-frame time)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5f
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5f/pytest.log 2>&1 || { tail -30 gpurun_out/r5f/pytest.log; exit 1; }
tail -2 gpurun_out/r5f/pytest.log
timeout -k 10 300 python bench.py > gpurun_out/r5f/bench.json 2> gpurun_out/r5f/bench.err || { tail -20 gpurun_out/r5f/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r5f/bench.json'));print(d['value'], d['ms_per_step'], d['config']['scratch'], d['single_frame']['kernel_ms'], d['moving_camera']['kernel_ms_per_frame'], d['also'])"
timeout -k 10 300 python bench.py --workload synth10k_3840x2160_d6 --steps 16 --warmup 8 --no-also --no-cpu-baseline --no-extras > gpurun_out/r5f/bench_synth10k.json 2> gpurun_out/r5f/bench_synth10k.err || { tail -20 gpurun_out/r5f/bench_synth10k.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r5f/bench_synth10k.json'));print(d['value'], d['ms_per_step'], d['config']['scratch'])"
