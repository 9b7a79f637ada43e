#!/usr/bin/env bash
# round-5 session o: wave-wide broadcast neighbour scan in the single-workgroup build: phases, drift, TLAS tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05o}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_inflight.py -m gpu -q -rs --timeout 150 --timeout-method thread -k "long_motion or moving_instances or materials or in_flight or many_inst or tlas" > gpurun_out/${T}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times.log 2>&1 || exit $?
grep "small build" gpurun_out/${T}_times.log | tail -2
for k in 1 2; do
  TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_$k.log 2>&1 || exit $?
  grep instances gpurun_out/${T}_drift_$k.log
done
exit $rc
