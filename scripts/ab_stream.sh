# streaming engine: parity against the wavefront, then rank-0 shares (C4) with PRT_STREAM=1 vs 0
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "streaming" > gpurun_out/tg_stream.log 2>&1; rc=$?
tail -30 gpurun_out/tg_stream.log
[ $rc -eq 0 ] || exit $rc
for s in 1 0; do
  echo "== PRT_STREAM=$s"
  PRT_STREAM=$s timeout -k 10 300 python scripts/rank_time.py ${WORLDS:-8 4 2 1} > gpurun_out/rank_s$s.log 2>&1 || { tail -5 gpurun_out/rank_s$s.log; exit 1; }
  grep world gpurun_out/rank_s$s.log
done
