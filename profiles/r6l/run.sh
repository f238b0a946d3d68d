# light grids: spheres within a shadow ray's EPSILON overshoot of a light on its global list
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6l
# the new scene against the previous build (expected to differ from the oracle) -- the test catches the defect
RT_HIP_LIB="$GRAFT_REPO_ROOT/build_variants/librt_hip_r5y.so" timeout -k 10 300 python -u -m pytest tests/test_light_grid.py -q -k "sphere_beyond_light" -m gpu --timeout 120 --timeout-method thread > gpurun_out/r6l/old_build_new_scene.log 2>&1; echo "old build rc $? (nonzero expected)"
tail -3 gpurun_out/r6l/old_build_new_scene.log | cut -c1-300
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6l/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r6l/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6l/pytest_gpu.log
timeout -k 10 120 python -u scripts/fuzz_repro.py 7101 4787 > gpurun_out/r6l/repro.log 2>&1 || exit 1
grep "three positions, rep 0\|single" gpurun_out/r6l/repro.log | cut -c1-200
timeout -k 10 400 python -u scripts/gpu_fuzz.py 330 7101 > gpurun_out/r6l/fuzz_7101.log 2>&1 || { tail -3 gpurun_out/r6l/fuzz_7101.log; exit 1; }
tail -1 gpurun_out/r6l/fuzz_7101.log
