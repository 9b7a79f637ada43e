#!/usr/bin/env bash
# round-5 session e: GPU suite, instance-BVH drift (pipelined single-workgroup rebuild), kernel traces of the
# drift and of the world-8 share with 2 / 3 frames in flight
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05e}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 150 --timeout-method thread \
  > gpurun_out/${T}_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/${T}_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 600 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift.log 2>&1 || exit $?
cat gpurun_out/${T}_drift.log
TLAS_MODES=default timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_drift_trace -o run -- \
  python3 scripts/tlas_drift.py 1000 40 > gpurun_out/${T}_drift_trace.log 2>&1 || { tail -5 gpurun_out/${T}_drift_trace.log; exit 1; }
f=$(find gpurun_out/${T}_drift_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$f" --focus k_build_small | tee gpurun_out/${T}_drift_timeline.txt
for fl in 2 3; do
  PRT_RANK_INFLIGHT=$fl timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_w8_fl$fl -o run -- \
    python3 scripts/rank_time.py 8 > gpurun_out/${T}_w8_fl$fl.log 2>&1 || { tail -5 gpurun_out/${T}_w8_fl$fl.log; exit 1; }
  grep world gpurun_out/${T}_w8_fl$fl.log
  f=$(find gpurun_out/${T}_w8_fl$fl -name "*kernel_trace.csv" | head -1)
  python3 scripts/timeline.py "$f" --focus none | head -4
done
exit $rc
