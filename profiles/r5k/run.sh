# (1) round-4 library vs current on the driver's 20/5 protocol, same box, alternating;
# (2) cfg 5 with the decoupled grid-walk deferred kernel; (3) fuzz of it (every scene on the uniform grid)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5k
SKIP_TESTS=1 REPS=3 TAG=r5k/ab20 LIBS="build_variants/librt_hip_r4.so cur" BENCH_ARGS="--steps 20 --warmup 5 --no-extras" bash scripts/gpu_libab.sh > gpurun_out/r5k/ab_r4_vs_cur_20_5.log 2>&1 || { tail -20 gpurun_out/r5k/ab_r4_vs_cur_20_5.log; exit 1; }
cat gpurun_out/r5k/ab_r4_vs_cur_20_5.log
timeout -k 10 600 python -u scripts/ab_launch.py "default;RT_HIP_DEFER_GRID=1;RT_HIP_DEFER_GRID=1+RT_HIP_DEFER_LEVEL=1+RT_HIP_DEFER_DIV=2" synth10k_3840x2160_d6 > gpurun_out/r5k/ab_defer_grid.log 2>&1 || { tail -20 gpurun_out/r5k/ab_defer_grid.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5k/ab_defer_grid.log
FUZZ_VARIANT=tuning RT_HIP_DEFER_GRID=1 RT_HIP_BEHIND_GRID=1 RT_HIP_BVH_ALWAYS=1 timeout -k 10 200 python -u scripts/gpu_fuzz.py 170 23 > gpurun_out/r5k/fuzz_defer_grid.log 2>&1 || { tail -5 gpurun_out/r5k/fuzz_defer_grid.log; exit 1; }
tail -1 gpurun_out/r5k/fuzz_defer_grid.log
