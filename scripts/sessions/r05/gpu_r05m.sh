#!/usr/bin/env bash
# round-5 session m: bench.py frames in flight 2 vs 4 at N = 1 (C4, interleaved) and C5 one at a time vs 2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05m}
bench() {  # bench <tag> <args...>
  local t=$1; shift
  timeout -k 10 300 python bench.py --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${T}_$t.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['config']['frames_in_flight'], d['config']['hw_queues'])" gpurun_out/${T}_$t.log $t
}
for r in 1 2 3; do
  bench c4_fl2_$r --steps 20 --inflight 2
  bench c4_fl4_$r --steps 20 --inflight 4
done
bench c5_fl1 --scene c5 --steps 3 --inflight 1
bench c5_fl2 --scene c5 --steps 3 --inflight 2
