#!/usr/bin/env bash
# round-5 session d: kernel timeline of the default instance-BVH rebuild during drift; frames-in-flight grid A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05d}
TLAS_MODES=default timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_drift_trace -o run -- \
  python3 scripts/tlas_drift.py 1000 40 > gpurun_out/${T}_drift_trace.log 2>&1 || { tail -5 gpurun_out/${T}_drift_trace.log; exit 1; }
tail -2 gpurun_out/${T}_drift_trace.log
f=$(find gpurun_out/${T}_drift_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$f" --focus k_build_small | tee gpurun_out/${T}_drift_timeline.txt
for g in 1 2 4; do for fl in 2 3; do
  PRT_FLIGHT_GRID=$g PRT_RANK_INFLIGHT=$fl timeout -k 10 300 python -u scripts/rank_time.py 1 8 > gpurun_out/${T}_rank_g${g}_fl$fl.log 2>&1 || exit $?
  echo "grid 1/$g"; grep world gpurun_out/${T}_rank_g${g}_fl$fl.log
done; done
for fl in 2 3; do
  PRT_MERGE=0 PRT_RANK_INFLIGHT=$fl timeout -k 10 300 python -u scripts/rank_time.py 8 > gpurun_out/${T}_rank_nomerge_fl$fl.log 2>&1 || exit $?
  echo "unmerged"; grep world gpurun_out/${T}_rank_nomerge_fl$fl.log
done
