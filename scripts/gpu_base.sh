# baseline: bench (N=1) + rank-0 shares at world 1/2/4/8, each under its own limit
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 python scripts/rank_time.py > gpurun_out/rank.log 2>&1 || { tail -20 gpurun_out/rank.log; exit 1; }
grep world gpurun_out/rank.log
