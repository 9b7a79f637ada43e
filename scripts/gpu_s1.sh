# session 1: changed GPU tests, bench, rank-0 shares (1 / 2 / 4 concurrent item groups), lane-usage histogram,
# instance-BVH drift
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_checkpoint.py tests/test_gpu_parity.py -k "shard or checkpoint or groups or pass_limit or failed or tlas" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -40 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
bash scripts/gpu_base.sh || exit $?
for g in 2 4; do
  PRT_GROUPS=$g timeout -k 10 300 python scripts/rank_time.py > gpurun_out/rank_g$g.log 2>&1 || { tail -20 gpurun_out/rank_g$g.log; exit 1; }
  echo "groups $g"; grep world gpurun_out/rank_g$g.log
done
timeout -k 10 400 python scripts/tlas_drift.py 1000 200 > gpurun_out/drift.log 2>&1 || { tail -20 gpurun_out/drift.log; exit 1; }
cat gpurun_out/drift.log
bash scripts/gpu_lanestats.sh r04 || exit $?
