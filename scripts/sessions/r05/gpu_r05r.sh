#!/usr/bin/env bash
# round-5 session r: instance-BVH build split (PLOC kernel + 256-thread collapse kernel with the tree in LDS),
# 256-thread finish / commit / refit kernels, vectorised drift host loop; radius 512 vs 64; in-place updates
# (DRIFT_VEL=0) against the static frame; kernel timeline of 40 drifting frames
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05r}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_inflight.py -m gpu -q -rs --timeout 150 --timeout-method thread -k "long_motion or moving_instances or materials or instance or flight" > gpurun_out/${T}_tlas_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tlas_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tlas_tests.log
for r in 512 64; do
  PRT_TLAS_SMALL_R=$r PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times_r$r.log 2>&1 || exit $?
  echo "radius $r"; grep "small build" gpurun_out/${T}_times_r$r.log | tail -2
done
for k in 1 2; do
  for cfg in "512 1" "64 1" "512 0"; do
    set -- $cfg
    DRIFT_VEL=$2 PRT_TLAS_SMALL_R=$1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_r$1_v$2_$k.log 2>&1 || exit $?
    echo "radius $1 vel $2"; grep instances gpurun_out/${T}_drift_r$1_v$2_$k.log
  done
done
TLAS_MODES=default timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_drift_trace -o run -- \
  python3 scripts/tlas_drift.py 1000 40 > gpurun_out/${T}_drift_trace.log 2>&1 || { tail -5 gpurun_out/${T}_drift_trace.log; exit 1; }
f=$(find gpurun_out/${T}_drift_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$f" --focus k_build_small > gpurun_out/${T}_drift_timeline.txt && cat gpurun_out/${T}_drift_timeline.txt
