#!/usr/bin/env bash
# round-5 session q: wave-per-cluster incremental neighbour search in the single-workgroup instance-BVH build;
# PLOC radius sweep (phase clock + drift, 1,000 instances); the instance-BVH tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05q}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_inflight.py -m gpu -q -rs --timeout 150 --timeout-method thread -k "long_motion or moving_instances or materials or instance or flight" > gpurun_out/${T}_tlas_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tlas_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tlas_tests.log
for r in 512 128 64 32; do
  PRT_TLAS_SMALL_R=$r PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times_r$r.log 2>&1 || exit $?
  echo "radius $r"; grep "small build" gpurun_out/${T}_times_r$r.log | tail -2
done
for r in 512 64 512 64; do
  PRT_TLAS_SMALL_R=$r TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_r$r.log 2>&1 || exit $?
  echo "radius $r"; grep instances gpurun_out/${T}_drift_r$r.log
done
