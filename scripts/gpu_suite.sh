#!/usr/bin/env bash
# The whole GPU parity suite on the library in the tree, time-limited; log under gpurun_out/<tag>_gpu.log
#   scripts/gpu_suite.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-suite}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/${T}_gpu.log
exit $rc
