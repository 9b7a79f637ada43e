#!/usr/bin/env bash
# round-5 session v: the instance-BVH build launches holding their CU's whole LDS (PRT_TLAS_FULL_CU 1 / 0), drift;
# kernel timeline of 40 drifting frames
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05v}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rs --timeout 150 --timeout-method thread -k "long_motion or moving_instances or materials" > gpurun_out/${T}_tlas_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tlas_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tlas_tests.log
PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times.log 2>&1 || exit $?
grep "prt: small build" gpurun_out/${T}_times.log | tail -3
for k in 1 2 3; do
  for f in 1 0; do
    PRT_TLAS_FULL_CU=$f TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_f${f}_$k.log 2>&1 || exit $?
    echo "full CU $f"; grep instances gpurun_out/${T}_drift_f${f}_$k.log
  done
done
TLAS_MODES=default timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_drift_trace -o run -- \
  python3 scripts/tlas_drift.py 1000 40 > gpurun_out/${T}_drift_trace.log 2>&1 || { tail -5 gpurun_out/${T}_drift_trace.log; exit 1; }
f=$(find gpurun_out/${T}_drift_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$f" --focus k_build_small > gpurun_out/${T}_drift_timeline.txt && cat gpurun_out/${T}_drift_timeline.txt
