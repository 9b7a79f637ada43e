#!/usr/bin/env bash
# round-5 session s: reserved build CU (PRT_BUILD_CU 1 / 0) for the single-workgroup instance-BVH build; radius
# 512 / 64; in-place updates (DRIFT_VEL=0); phase clock
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05s}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_inflight.py -m gpu -q -rs --timeout 150 --timeout-method thread -k "long_motion or moving_instances or materials or instance or flight" > gpurun_out/${T}_tlas_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tlas_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tlas_tests.log
for cu in 1 0; do
  PRT_BUILD_CU=$cu PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times_cu$cu.log 2>&1 || exit $?
  echo "build CU $cu"; grep "small build" gpurun_out/${T}_times_cu$cu.log | tail -2
done
for k in 1 2; do
  for cfg in "1 512 1" "0 512 1" "1 64 1" "1 512 0"; do
    set -- $cfg
    PRT_BUILD_CU=$1 DRIFT_VEL=$3 PRT_TLAS_SMALL_R=$2 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_cu$1_r$2_v$3_$k.log 2>&1 || exit $?
    echo "build CU $1 radius $2 vel $3"; grep instances gpurun_out/${T}_drift_cu$1_r$2_v$3_$k.log
  done
done
