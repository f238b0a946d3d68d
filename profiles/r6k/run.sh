# the fuzz mismatch on diagnostic builds: no shadow-line bound, no root-free decisions
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6k
for v in nooff noroot; do
  RT_HIP_LIB="$GRAFT_REPO_ROOT/build_variants/librt_hip_$v.so" timeout -k 10 120 python -u scripts/fuzz_repro.py 7101 4787 > gpurun_out/r6k/repro_$v.log 2>&1; echo "$v rc $?"
  grep -v amdgpu.ids gpurun_out/r6k/repro_$v.log | grep "single\|three positions, rep 0" | cut -c1-300
done
