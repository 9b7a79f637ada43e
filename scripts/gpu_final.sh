#!/usr/bin/env bash
# End-of-round GPU session: smoke + GPU suite + bench (with the CPU baseline), then the stamped rocprofv3 passes
# (kernel stats, FETCH_SIZE, WRITE_SIZE, VALU), rank-0 shares at world 1/2/4/8 and a C5 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_check.sh all || exit $?
bash scripts/gpu_check.sh prof || exit $?
timeout -k 10 300 python scripts/rank_time.py > gpurun_out/rank_final.log 2>&1 || exit $?
grep world gpurun_out/rank_final.log
timeout -k 10 300 python bench.py --scene c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c5.log
