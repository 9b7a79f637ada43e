set -o pipefail
mkdir -p gpurun_out
REPS=4 timeout -k 10 120 python scripts/stream_diag.py > gpurun_out/diag.log 2>&1 || { tail -5 gpurun_out/diag.log; exit 1; }
grep -c "differing pixels 0 " gpurun_out/diag.log; grep rep gpurun_out/diag.log | grep -v "differing pixels 0 " | head -5
for uc in 0 1; do
  echo "== PRT_STREAM_UC=$uc"
  PRT_STREAM=1 PRT_STREAM_UC=$uc timeout -k 10 300 python scripts/rank_time.py 8 1 > gpurun_out/rank_uc$uc.log 2>&1 || { tail -5 gpurun_out/rank_uc$uc.log; exit 1; }
  grep world gpurun_out/rank_uc$uc.log
done
