# session 12: the full GPU suite on the new defaults (shading kernel ray prefetch, dense resolve, sync-free
# single-workgroup instance-BVH rebuild), then the 1,000-instance drift (refit only / trigger / every frame)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s12_tests.log 2>&1; rc=$?
tail -5 gpurun_out/s12_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/s12_tests.log | head -30; exit $rc; }
timeout -k 10 280 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/drift12.log 2>&1; rc=$?
grep instances gpurun_out/drift12.log
exit $rc
