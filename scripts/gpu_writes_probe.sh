# Where the render kernel's HBM writes come from (round 6): PMC WRITE_SIZE of
# the synth200 bench launches on the tuning build under knob settings.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$ROOT"
OUT=gpurun_out/r7g; mkdir -p $OUT
export TMPDIR=/tmp
export RT_HIP_LIB=$ROOT/cs420-ray-tracer_amd/variants/librt_hip_tuning.so
i=0
for knobs in "X=1" "RT_HIP_DEFER=0" "RT_HIP_WIDE=0" "RT_HIP_DEFER=0 RT_HIP_WIDE=0" "RT_HIP_CAM_GRID=0" "RT_HIP_SPHERE_GRID=0"; do
  ( export $knobs; timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p$i -o run -- python3 bench.py --no-cpu-baseline --no-also --no-extras --workload synth200_1920x1080_d4 --steps 32 --warmup 16 > $OUT/p$i.log 2>&1 ) || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "$i $knobs" >> $OUT/passes.txt
  i=$((i+1))
done
