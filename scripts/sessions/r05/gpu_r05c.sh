#!/usr/bin/env bash
# round-5 session c: GPU suite on the library with up to 4 frames in flight and the single-workgroup instance-BVH
# rebuild as the default, then rank shares / bench per frames in flight and the instance-BVH drift
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05c}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 150 --timeout-method thread \
  > gpurun_out/${T}_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/${T}_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
for fl in 1 2 3 4; do
  PRT_RANK_INFLIGHT=$fl timeout -k 10 300 python -u scripts/rank_time.py 1 8 > gpurun_out/${T}_rank_fl$fl.log 2>&1 || exit $?
  grep world gpurun_out/${T}_rank_fl$fl.log
done
bench() {  # bench <tag> <args...>
  local t=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${T}_$t.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_ms'])" gpurun_out/${T}_$t.log $t
}
for r in 1 2; do for fl in 1 2 3 4; do bench fl${fl}_$r --inflight $fl; done; done
timeout -k 10 600 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/${T}_drift.log 2>&1 || exit $?
cat gpurun_out/${T}_drift.log
exit $rc
