#!/usr/bin/env bash
# round-5 session ac: instance-BVH buffers sized for n nodes under the per-update host build (no reallocation);
# the whole GPU suite; drift default (all policies once)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05ac}
bash scripts/gpu_suite.sh $T || exit $?
for k in 1 2; do
  TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_default_$k.log 2>&1 || exit $?
  grep instances gpurun_out/${T}_drift_default_$k.log
done
timeout -k 10 600 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_all.log 2>&1 || exit $?
grep instances gpurun_out/${T}_drift_all.log
