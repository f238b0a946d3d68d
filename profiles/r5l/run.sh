# same-box A/B at the driver's 20/5: round-4 library, round 5 before the bounded stacks (dbca82d), current;
# then row-shard probes: 20-frame launches at G = 1, 8 with and without deferral, one-frame complex at G = 8
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5l
SKIP_TESTS=1 REPS=4 TAG=r5l/ab20 LIBS="build_variants/librt_hip_r4.so build_variants/librt_hip_r5sg.so cur" BENCH_ARGS="--steps 20 --warmup 5 --no-extras" bash scripts/gpu_libab.sh > gpurun_out/r5l/ab_20_5.log 2>&1 || { tail -20 gpurun_out/r5l/ab_20_5.log; exit 1; }
cat gpurun_out/r5l/ab_20_5.log
PROBE_VARIANT=tuning FPL=20 GS=1,8 timeout -k 10 300 python scripts/shard_probe.py synth200_1920x1080_d4 4 > gpurun_out/r5l/shard20_defer.json 2>/dev/null || exit 1
PROBE_VARIANT=tuning RT_HIP_DEFER=0 FPL=20 GS=1,8 timeout -k 10 300 python scripts/shard_probe.py synth200_1920x1080_d4 4 > gpurun_out/r5l/shard20_nodefer.json 2>/dev/null || exit 1
FPL=1 GS=1,2,4,8 timeout -k 10 300 python scripts/shard_probe.py complex_1920x1080_d4 20 > gpurun_out/r5l/shard1_complex.json 2>/dev/null || exit 1
cat gpurun_out/r5l/shard20_defer.json gpurun_out/r5l/shard20_nodefer.json gpurun_out/r5l/shard1_complex.json
