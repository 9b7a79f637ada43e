#!/usr/bin/env bash
# The whole GPU parity suite on the library in the tree, then the single-workgroup instance-BVH builder's opt-in
# test modes (PRT_TEST_TLAS_SMALL=1), each step time-limited; logs under gpurun_out/
#   scripts/gpu_suite.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-suite}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 150 --timeout-method thread \
  > gpurun_out/${T}_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/${T}_gpu.log
# a fault, abort or time limit ends the call here; ordinary test failures go on to the small-builder modes
case $rc in 0|1) ;; *) exit $rc ;; esac
PRT_TEST_TLAS_SMALL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rs --timeout 150 \
  --timeout-method thread -k "long_motion and small" > gpurun_out/${T}_small.log 2>&1; rc2=$?
tail -8 gpurun_out/${T}_small.log
[ $rc -eq 0 ] && exit $rc2
exit $rc
