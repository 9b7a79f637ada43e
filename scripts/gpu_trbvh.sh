#!/usr/bin/env bash
# Treelet restructuring of the device builders (PRT_TRBVH passes): the builder parity test with it on, then build
# time and C4 / Spaceship rate for 0..3 passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PRT_TRBVH=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "builder" > gpurun_out/trbvh_tests.log 2>&1 || { tail -30 gpurun_out/trbvh_tests.log; exit 1; }
tail -1 gpurun_out/trbvh_tests.log
for t in 0 1 2 3; do
  for s in c4 ship; do
    PRT_TRBVH=$t timeout -k 10 300 python scripts/build_time.py only-gpu $s > "gpurun_out/trbvh_${t}_$s.log" 2>&1 || exit $?
    grep GPU "gpurun_out/trbvh_${t}_$s.log" | sed "s/^/T$t $s: /"
  done
done
