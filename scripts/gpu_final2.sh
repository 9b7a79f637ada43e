# final-build check: GPU suite, smoke, bench (N=1), rank-0 shares (two runs), world-8 timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/tg.log 2>&1 || { tail -40 gpurun_out/tg.log; exit 1; }
tail -2 gpurun_out/tg.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 python scripts/rank_time.py > gpurun_out/rank.log 2>&1 || exit $?
timeout -k 10 300 python scripts/rank_time.py > gpurun_out/rank2.log 2>&1 || exit $?
grep world gpurun_out/rank.log gpurun_out/rank2.log
rm -rf gpurun_out/w8
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/w8 -o run -- python3 scripts/rank_time.py 8 > gpurun_out/w8.log 2>&1 || exit $?
f=$(find gpurun_out/w8 -name '*kernel_trace.csv' | head -1)
python3 scripts/frame_timeline.py "$f" > gpurun_out/w8_timeline.txt && tail -3 gpurun_out/w8_timeline.txt
