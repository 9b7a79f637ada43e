# world-8 rank share and launch timeline with and without the cooperative traversal tail
set -o pipefail
mkdir -p gpurun_out
for t in 1 0; do
  echo "== PRT_TAIL=$t"
  PRT_TAIL=$t timeout -k 10 200 python scripts/rank_time.py 1 8 > gpurun_out/rank_tail$t.log 2>&1 || exit $?
  grep world gpurun_out/rank_tail$t.log
  PRT_TAIL=$t PRT_DEBUG_QUEUES=1 timeout -k 10 200 python scripts/rank_time.py 8 > gpurun_out/tl_tail$t.log 2>&1 || exit $?
  grep -E "trace [0-9]|iteration" gpurun_out/tl_tail$t.log | tail -18
done
PRT_DEBUG_QUEUES=1 timeout -k 10 200 python scripts/rank_time.py 1 > gpurun_out/tl_w1.log 2>&1 || exit $?
grep -E "trace [0-9]|iteration" gpurun_out/tl_w1.log | tail -18
