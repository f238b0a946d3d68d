# A long randomised parity campaign on the final tree (new seeds, every
# generator; SET=2: large images and the bounds-checked build; SET=3: the
# product's environment knobs; SET=4: the tuning build's other layouts): scripts/gpu_fuzz.py
# phases of $SECS seconds each; stops at the
# first mismatch (the scene goes to gpurun_out/fuzz_mismatch.txt).
set -o pipefail
OUT=gpurun_out/fuzz_campaign; mkdir -p $OUT; export TMPDIR=/tmp
SECS=${SECS:-240}; B=${SEED_BASE:-5100}
run() { name=$1; shift; timeout -k 10 $((SECS + 60)) env "$@" python -u scripts/gpu_fuzz.py $SECS $((B + ${#name})) > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }; echo "$name: $(tail -1 $OUT/$name.log)"; }
if [ "${SET:-1}" = 1 ]; then
  run general FUZZ_X=0
  run near_lights FUZZ_NEAR_LIGHTS=1
  run margin FUZZ_MARGIN=1
  run margin_camgrid FUZZ_MARGIN=1 RT_HIP_CAM_GRID=2
elif [ "$SET" = 2 ]; then  # images of 1,024+ tiles (tile order, launch tails, deferral shards) and the bounds-checked build
  run large_general FUZZ_LARGE=1
  run large_near_lights FUZZ_LARGE=1 FUZZ_NEAR_LIGHTS=1
  run checked_margin FUZZ_MARGIN=1 FUZZ_VARIANT=check
  run checked_general FUZZ_VARIANT=check
elif [ "$SET" = 4 ]; then  # the tuning build's other layouts (test-only paths sharing the product's code)
  run t_global_stack FUZZ_VARIANT=tuning RT_HIP_STACK=1
  run t_nodefer_nosched FUZZ_VARIANT=tuning RT_HIP_DEFER=0 RT_HIP_SCHED=0 RT_HIP_WIDE=0
  run t_grid_forced FUZZ_MARGIN=1 FUZZ_VARIANT=tuning RT_HIP_BEHIND_GRID=1 RT_HIP_BVH_ALWAYS=1 RT_HIP_SPHERE_GRID=0
  run t_bvh2_walk FUZZ_VARIANT=tuning RT_HIP_BVH4=0 RT_HIP_BVH_ALWAYS=1 RT_HIP_DEFER_LEVEL=1 RT_HIP_MERGE_Q=8
else  # the product library's two environment knobs: the LDS-staged scene, the camera grid off / every launch
  run lds_general RT_HIP_LDS_SCENE=1
  run lds_margin FUZZ_MARGIN=1 RT_HIP_LDS_SCENE=1
  run camgrid0_near FUZZ_NEAR_LIGHTS=1 RT_HIP_CAM_GRID=0
  run camgrid2_general RT_HIP_CAM_GRID=2
fi
