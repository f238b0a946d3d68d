#!/bin/bash
# One GPU session: smoke, parity tests, CLI timing.  Stops at the first crash-like exit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
cd cs420-ray-tracer_amd
for cfg in "complex 1920 1080 4" "synth200 1920 1080 4" "medium 1920 1080 2" "simple 800 600 10"; do
  set -- $cfg
  timeout -k 10 120 ./ray_hip scenes/$1.txt --width $2 --height $3 --depth $4 --repeat 5 --json --p6 --out ../gpurun_out/$1_$2x$3.ppm > ../gpurun_out/cli_$1.log 2>&1; rc=$?
  echo "cli $1 rc=$rc"; grep -E "^\{|time" ../gpurun_out/cli_$1.log
  [ $rc -eq 0 ] || exit $rc
done
