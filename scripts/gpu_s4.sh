# session 4: async device TLAS rebuild (test + drift), then the triangle-pool A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "tlas" > gpurun_out/t4.log 2>&1 || { tail -30 gpurun_out/t4.log; exit 1; }
tail -2 gpurun_out/t4.log
timeout -k 10 500 python scripts/tlas_drift.py 1000 200 > gpurun_out/drift.log 2>&1 || { tail -20 gpurun_out/drift.log; exit 1; }
cat gpurun_out/drift.log
bash scripts/gpu_pool_ab.sh pool88
