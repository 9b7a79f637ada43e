#!/usr/bin/env bash
# round-5 session x: collapse octant assignment from precomputed centroid offsets, workgroup-scope DP table in the
# single-workgroup build; the whole GPU suite, phase clock, drift
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05x}
bash scripts/gpu_suite.sh $T || exit $?
PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times.log 2>&1 || exit $?
grep "small build n=" gpurun_out/${T}_times.log | tail -2
for k in 1 2 3; do
  TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_$k.log 2>&1 || exit $?
  grep instances gpurun_out/${T}_drift_$k.log
done
timeout -k 10 300 python -u scripts/build_time.py > gpurun_out/${T}_build_time.log 2>&1; tail -5 gpurun_out/${T}_build_time.log
