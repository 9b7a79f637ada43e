# GPU parity suite (optionally filtered by -k), then a short bench; every GPU step time-limited
set -o pipefail
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/tg.log 2>&1; rc=$?
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/tg.log 2>&1; rc=$?
fi
tail -30 gpurun_out/tg.log
[ $rc -eq 0 ] || exit $rc
if [ -n "${2:-}" ]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline $2 > gpurun_out/bench_t.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_t.log
fi
