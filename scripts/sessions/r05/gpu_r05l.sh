#!/usr/bin/env bash
# round-5 session l: octant-ordered next-ray appends (PRT_SORT_OCT) A/B with parity; 4-in-flight default grids
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05l}
PRT_SORT_OCT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_golden_ref.py -m gpu -q -rs --timeout 150 --timeout-method thread > gpurun_out/${T}_sort_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_sort_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
bench() {  # bench <tag> <args...>
  local t=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${T}_$t.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_ms'])" gpurun_out/${T}_$t.log $t
}
for r in 1 2; do
  PRT_SORT_OCT=0 bench s0_fl1_$r --inflight 1
  PRT_SORT_OCT=1 bench s1_fl1_$r --inflight 1
  PRT_SORT_OCT=0 bench s0_fl2_$r
  PRT_SORT_OCT=1 bench s1_fl2_$r
done
GPU_MAX_HW_QUEUES=8 PRT_RANK_INFLIGHT=4 timeout -k 10 300 python -u scripts/rank_time.py 1 2 4 8 > gpurun_out/${T}_rank_fl4.log 2>&1 || exit $?
grep world gpurun_out/${T}_rank_fl4.log
exit $rc
