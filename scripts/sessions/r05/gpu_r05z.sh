#!/usr/bin/env bash
# round-5 session z: are the slow traversal launches of the drift the rebuild's?  Kernel traces of 40 drifting
# frames with the default device rebuild and with a host SAH build per update, and of 40 static frames
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05z}
for m in default host; do
  TLAS_MODES=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_${m}_trace -o run -- \
    python3 scripts/tlas_drift.py 1000 60 > gpurun_out/${T}_${m}_trace.log 2>&1 || { tail -5 gpurun_out/${T}_${m}_trace.log; exit 1; }
  f=$(find gpurun_out/${T}_${m}_trace -name "*kernel_trace.csv" | head -1)
  echo "== $m"; grep instances gpurun_out/${T}_${m}_trace.log
  python3 scripts/timeline.py "$f" --focus k_build_small > gpurun_out/${T}_${m}_timeline.txt && tail -3 gpurun_out/${T}_${m}_timeline.txt
done
