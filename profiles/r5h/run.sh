# deferred-queue room / level A/B (cfg 5 and the metric), the one-frame tail length, and a kernel trace of the synth10k bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5h
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/ab_launch.py "default;RT_HIP_DEFER_DIV=16;RT_HIP_DEFER_DIV=32;RT_HIP_DEFER_DIV=4;RT_HIP_DEFER_LEVEL=3" synth10k_3840x2160_d6 synth200_1920x1080_d4 > gpurun_out/r5h/ab_defer.log 2>&1 || { tail -20 gpurun_out/r5h/ab_defer.log; exit 1; }
timeout -k 10 400 python -u scripts/ab_launch.py "default;RT_HIP_TAIL_WAVES=6;RT_HIP_TAIL_WAVES=24;RT_HIP_TAIL_WAVES=36" synth200_1920x1080_d4 complex_1920x1080_d4 > gpurun_out/r5h/ab_tail.log 2>&1 || { tail -20 gpurun_out/r5h/ab_tail.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5h/trace10k -o run -- python3 bench.py --workload synth10k_3840x2160_d6 --steps 16 --warmup 8 --no-also --no-cpu-baseline --no-extras > gpurun_out/r5h/trace10k_bench.json 2> gpurun_out/r5h/trace10k_bench.err || { tail -5 gpurun_out/r5h/trace10k_bench.err; exit 1; }
head -12 gpurun_out/r5h/trace10k/run_kernel_stats.csv
