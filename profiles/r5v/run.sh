# round profile on the current sources, then the driver's 20/5 line against 64/16, alternating
cd "$GRAFT_REPO_ROOT"
TAG=r5v bash scripts/gpu_profile.sh || exit 1
mkdir -p gpurun_out/r5v
for rep in 1 2 3; do
  for sw in "20 5" "64 16"; do
    set -- $sw
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-also --no-extras --steps $1 --warmup $2 > gpurun_out/r5v/bench_${1}_${2}_$rep.json 2> gpurun_out/r5v/bench_${1}_${2}_$rep.err || { tail -5 gpurun_out/r5v/bench_${1}_${2}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r5v/bench_${1}_${2}_$rep.json')); print('$1/$2', d['value'], d['ms_per_step'])"
  done
done
