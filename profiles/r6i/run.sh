# the fuzz mismatch (seed 7101, scene 4787) replayed with details: product, the r5y build, light lists by index
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6i
timeout -k 10 120 python -u scripts/fuzz_repro.py 7101 4787 > gpurun_out/r6i/repro_product.log 2>&1; echo "rc $?"
grep -v amdgpu.ids gpurun_out/r6i/repro_product.log | cut -c1-400
RT_HIP_LIB="$GRAFT_REPO_ROOT/build_variants/librt_hip_r5y.so" timeout -k 10 120 python -u scripts/fuzz_repro.py 7101 4787 > gpurun_out/r6i/repro_r5y.log 2>&1; echo "rc $?"
grep -v amdgpu.ids gpurun_out/r6i/repro_r5y.log | grep -v "^info" | cut -c1-300
FUZZ_VARIANT=tuning RT_HIP_LG_ORDER=0 timeout -k 10 120 python -u scripts/fuzz_repro.py 7101 4787 > gpurun_out/r6i/repro_lgorder0.log 2>&1; echo "rc $?"
grep -v amdgpu.ids gpurun_out/r6i/repro_lgorder0.log | grep -v "^info" | cut -c1-300
