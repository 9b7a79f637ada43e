#!/usr/bin/env bash
# round-5 session y: single-workgroup build PLOC radius 32 / 48 / 64 (phase clock, drift twice each, interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05y}
for r in 32 48 64; do
  PRT_TLAS_SMALL_R=$r PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times_r$r.log 2>&1 || exit $?
  echo "radius $r"; grep "small build n=" gpurun_out/${T}_times_r$r.log | tail -2
done
for k in 1 2; do
  for r in 32 48 64; do
    PRT_TLAS_SMALL_R=$r TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_r${r}_$k.log 2>&1 || exit $?
    echo "radius $r"; grep instances gpurun_out/${T}_drift_r${r}_$k.log
  done
done
