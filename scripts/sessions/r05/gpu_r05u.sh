#!/usr/bin/env bash
# round-5 session u: the whole GPU suite on the library with the radius-64 two-launch instance-BVH build; drift at
# the default (blocking commit) and pipelined; the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05u}
bash scripts/gpu_suite.sh $T || exit $?
PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times.log 2>&1 || exit $?
grep "small build" gpurun_out/${T}_times.log | tail -2
for k in 1 2; do
  for p in 0 1; do
    PRT_TLAS_PIPELINE=$p TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_p${p}_$k.log 2>&1 || exit $?
    echo "pipeline $p"; grep instances gpurun_out/${T}_drift_p${p}_$k.log
  done
done
timeout -k 10 600 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift_all.log 2>&1 || exit $?
cat gpurun_out/${T}_drift_all.log
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_bench.log | cut -c1-400
