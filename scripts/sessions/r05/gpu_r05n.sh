#!/usr/bin/env bash
# round-5 session n: bench.py at N = 1 with 2 / 4 frames in flight and 4 / 8 hardware queues; PLOC phase split
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05n}
bench() {  # bench <tag> <args...>
  local t=$1; shift
  timeout -k 10 300 python bench.py --warmup 2 --steps 20 --no-cpu-baseline "$@" > gpurun_out/${T}_$t.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['config']['frames_in_flight'], d['config']['hw_queues'])" gpurun_out/${T}_$t.log $t
}
for r in 1 2; do
  bench fl2_q4_$r --inflight 2
  GPU_MAX_HW_QUEUES=8 bench fl2_q8_$r --inflight 2
  bench fl4_q8_$r --inflight 4
done
PRT_TLAS_SMALL_TIMES=1 TLAS_MODES=default timeout -k 10 300 python -u scripts/tlas_drift.py 1000 20 > gpurun_out/${T}_times.log 2>&1 || exit $?
grep "small build" gpurun_out/${T}_times.log | tail -2
