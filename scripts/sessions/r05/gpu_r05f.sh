#!/usr/bin/env bash
# round-5 session f: the single-workgroup build's phase times per PLOC radius, drift per radius; frames in flight
# with more hardware queues
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05f}
for r in 512 128 64 32; do
  PRT_TLAS_SMALL_R=$r PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 \
    > gpurun_out/${T}_times_r$r.log 2>&1 || exit $?
  echo "radius $r"; grep "small build" gpurun_out/${T}_times_r$r.log | tail -3
done
for r in 512 64; do
  PRT_TLAS_SMALL_R=$r TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 100 > gpurun_out/${T}_drift_r$r.log 2>&1 || exit $?
  echo "radius $r"; grep instances gpurun_out/${T}_drift_r$r.log
done
for fl in 2 3 4; do
  GPU_MAX_HW_QUEUES=8 PRT_RANK_INFLIGHT=$fl timeout -k 10 300 python -u scripts/rank_time.py 1 8 > gpurun_out/${T}_rank_q8_fl$fl.log 2>&1 || exit $?
  grep world gpurun_out/${T}_rank_q8_fl$fl.log
done
