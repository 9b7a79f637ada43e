#!/usr/bin/env bash
# round-5 session h: GPU suite (SoA single-workgroup build), build phases, frames in flight per world with 8 hardware
# queues, the bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05h}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 150 --timeout-method thread \
  > gpurun_out/${T}_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/${T}_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times.log 2>&1 || exit $?
grep "small build" gpurun_out/${T}_times.log | tail -3
for fl in 2 4; do
  GPU_MAX_HW_QUEUES=8 PRT_RANK_INFLIGHT=$fl timeout -k 10 300 python -u scripts/rank_time.py 1 2 4 8 > gpurun_out/${T}_rank_q8_fl$fl.log 2>&1 || exit $?
  grep world gpurun_out/${T}_rank_q8_fl$fl.log
done
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_bench.log
exit $rc
