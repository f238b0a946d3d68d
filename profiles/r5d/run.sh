# cfg 5 with sphere grids (device-built) instead of the uniform-grid walks for reflection rays: A/B + parity spot checks
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5d
timeout -k 10 600 python -u -m pytest tests/test_light_grid.py -x -q -k "sphere_grid" --timeout 300 --timeout-method thread > gpurun_out/r5d/pytest.log 2>&1 || { tail -30 gpurun_out/r5d/pytest.log; exit 1; }
tail -2 gpurun_out/r5d/pytest.log
timeout -k 10 900 python -u scripts/ab_launch.py "default;RT_HIP_SPHERE_GRID=1;RT_HIP_SPHERE_GRID=1+RT_HIP_SPHERE_GRID_N=32;RT_HIP_SPHERE_GRID=1+RT_HIP_SPHERE_GRID_N=8" synth10k_3840x2160_d6 > gpurun_out/r5d/ab_sg_synth10k.log 2>&1 || { tail -20 gpurun_out/r5d/ab_sg_synth10k.log; exit 1; }
cat gpurun_out/r5d/ab_sg_synth10k.log
