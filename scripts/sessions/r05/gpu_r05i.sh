#!/usr/bin/env bash
# round-5 session i: GPU suite (incremental PLOC neighbours, blocking commit by default), build phases, drift of the
# default / pipelined policies
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05i}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 150 --timeout-method thread \
  > gpurun_out/${T}_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/${T}_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times.log 2>&1 || exit $?
grep "small build" gpurun_out/${T}_times.log | tail -3
TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift.log 2>&1 || exit $?
grep instances gpurun_out/${T}_drift.log
PRT_TLAS_PIPELINE=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_pipe.log 2>&1 || exit $?
grep instances gpurun_out/${T}_drift_pipe.log
exit $rc
