#!/usr/bin/env bash
# round-5 session b: the GPU suite (+ small-builder modes), the frames-in-flight probe and A/Bs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05b}
bash scripts/gpu_suite.sh $T; rc=$?
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u scripts/inflight_probe.py 1 8 > gpurun_out/${T}_probe.log 2>&1 || exit $?
cat gpurun_out/${T}_probe.log
for fl in 1 2; do
  PRT_RANK_INFLIGHT=$fl timeout -k 10 300 python -u scripts/rank_time.py 1 2 4 8 > gpurun_out/${T}_rank_fl$fl.log 2>&1 || exit $?
  cat gpurun_out/${T}_rank_fl$fl.log
done
bench() {  # bench <tag> <args...>
  local t=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${T}_$t.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_ms'])" gpurun_out/${T}_$t.log $t
}
for r in 1 2; do
  PRT_OCC=7 bench occ7_fl1_$r --inflight 1
  PRT_OCC=8 bench occ8_fl1_$r --inflight 1
  PRT_OCC=7 bench occ7_fl2_$r --inflight 2
  PRT_OCC=8 bench occ8_fl2_$r --inflight 2
done
exit $rc
