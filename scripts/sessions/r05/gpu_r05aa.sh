#!/usr/bin/env bash
# round-5 session aa: the instance BVH rebuilt for every update by a builder thread (host SAH build beside the
# frames, taken by a later update) as the default; the whole GPU suite; drift default / device / host; timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05aa}
bash scripts/gpu_suite.sh $T || exit $?
for k in 1 2; do
  for m in default device host; do
    TLAS_MODES=$m timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_${m}_$k.log 2>&1 || exit $?
    echo "== $m"; grep instances gpurun_out/${T}_drift_${m}_$k.log
  done
done
TLAS_MODES=default timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_default_trace -o run -- \
  python3 scripts/tlas_drift.py 1000 60 > gpurun_out/${T}_default_trace.log 2>&1 || { tail -5 gpurun_out/${T}_default_trace.log; exit 1; }
f=$(find gpurun_out/${T}_default_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$f" > gpurun_out/${T}_default_timeline.txt && tail -2 gpurun_out/${T}_default_timeline.txt
timeout -k 10 600 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_all.log 2>&1 || exit $?
grep instances gpurun_out/${T}_drift_all.log
