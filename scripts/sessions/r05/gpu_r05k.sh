#!/usr/bin/env bash
# round-5 session k: traversal grid with one CU spare for the instance-BVH build, on the drift; world-8 share
# with 4 frames in flight and half grids
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05k}
for sp in 1 0 1 0; do
  PRT_SPARE_CU=$sp TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_spare$sp.log 2>&1 || exit $?
  echo "spare CU $sp"; grep instances gpurun_out/${T}_drift_spare$sp.log
done
PRT_FLIGHT_GRID=2 GPU_MAX_HW_QUEUES=8 PRT_RANK_INFLIGHT=4 timeout -k 10 300 python -u scripts/rank_time.py 1 8 > gpurun_out/${T}_rank_g2_fl4.log 2>&1 || exit $?
grep world gpurun_out/${T}_rank_g2_fl4.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_inflight.py -m gpu -q -rs --timeout 150 --timeout-method thread -k "long_motion or moving_instances or materials or in_flight" > gpurun_out/${T}_tests.log 2>&1; tail -3 gpurun_out/${T}_tests.log
