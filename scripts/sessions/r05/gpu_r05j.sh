#!/usr/bin/env bash
# round-5 session j: small-build PLOC radius (window vs global + incremental neighbours) and the depth slack, on
# the 1,000-instance drift; long-motion tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05j}
for r in 512 4096; do
  PRT_TLAS_SMALL_R=$r PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times_r$r.log 2>&1 || exit $?
  echo "radius $r"; grep "small build" gpurun_out/${T}_times_r$r.log | tail -2
done
for cfg in "512 1" "4096 1" "4096 auto"; do
  set -- $cfg
  PRT_TLAS_SMALL_R=$1 PRT_TLAS_SLACK=$2 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_r$1_$2.log 2>&1 || exit $?
  echo "radius $1 slack $2"; grep instances gpurun_out/${T}_drift_r$1_$2.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rs --timeout 150 --timeout-method thread -k "long_motion or moving_instances or materials" > gpurun_out/${T}_tlas_tests.log 2>&1; tail -3 gpurun_out/${T}_tlas_tests.log
