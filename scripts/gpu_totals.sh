# ray-totals change: GPU suite, smoke, bench (N=1, with CPU baseline), rank-0 shares; every GPU step time-limited
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/tg.log 2>&1 || { tail -40 gpurun_out/tg.log; exit 1; }
tail -3 gpurun_out/tg.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 python scripts/rank_time.py > gpurun_out/rank.log 2>&1 || exit $?
grep world gpurun_out/rank.log
timeout -k 10 300 python scripts/rank_time.py > gpurun_out/rank2.log 2>&1 || exit $?
grep world gpurun_out/rank2.log
