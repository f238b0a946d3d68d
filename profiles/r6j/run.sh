# the fuzz mismatch under knob settings (tuning build)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6j
timeout -k 10 300 python -u scripts/fuzz_repro.py 7101 4787 "default;RT_HIP_WIDE=0;RT_HIP_CAM_GRID=0;RT_HIP_SHADOW_GRID=0;RT_HIP_LG_ORDER=0;RT_HIP_SPHERE_GRID=0;RT_HIP_WIDE=0+RT_HIP_CAM_GRID=0" > gpurun_out/r6j/sweep.log 2>&1; echo "rc $?"
grep -v amdgpu.ids gpurun_out/r6j/sweep.log | cut -c1-600
