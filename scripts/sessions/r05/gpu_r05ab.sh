#!/usr/bin/env bash
# round-5 session ab: the host SAH build for every update as the default up to 4,096 instances; the whole GPU
# suite; drift default / device; kernel timeline of the default drift
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05ab}
bash scripts/gpu_suite.sh $T || exit $?
for k in 1 2 3; do
  for m in default device; do
    TLAS_MODES=$m timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_${m}_$k.log 2>&1 || exit $?
    echo "== $m"; grep instances gpurun_out/${T}_drift_${m}_$k.log
  done
done
TLAS_MODES=default timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_default_trace -o run -- \
  python3 scripts/tlas_drift.py 1000 60 > gpurun_out/${T}_default_trace.log 2>&1 || { tail -5 gpurun_out/${T}_default_trace.log; exit 1; }
f=$(find gpurun_out/${T}_default_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$f" > gpurun_out/${T}_default_timeline.txt && head -3 gpurun_out/${T}_default_timeline.txt && tail -1 gpurun_out/${T}_default_timeline.txt
