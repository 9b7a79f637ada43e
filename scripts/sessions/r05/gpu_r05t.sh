#!/usr/bin/env bash
# round-5 session t: instance-BVH rebuild policy under a host that keeps up (vectorised drift loop): committed at
# once vs one frame later (PRT_TLAS_PIPELINE), radius 512 / 64, spare CU 1 / 0; the collapse launch writes the
# instance slots and TlasMeta (no separate finish launch)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05t}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_inflight.py -m gpu -q -rs --timeout 150 --timeout-method thread -k "long_motion or moving_instances or materials or instance or flight" > gpurun_out/${T}_tlas_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tlas_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tlas_tests.log
PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times.log 2>&1 || exit $?
grep "small build" gpurun_out/${T}_times.log | tail -2
for k in 1 2; do
  for cfg in "0 512 1" "1 512 1" "0 64 1" "1 64 1" "0 512 0"; do
    set -- $cfg
    PRT_TLAS_PIPELINE=$1 PRT_TLAS_SMALL_R=$2 PRT_SPARE_CU=$3 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_p$1_r$2_s$3_$k.log 2>&1 || exit $?
    echo "pipeline $1 radius $2 spare $3"; grep instances gpurun_out/${T}_p$1_r$2_s$3_$k.log
  done
done
