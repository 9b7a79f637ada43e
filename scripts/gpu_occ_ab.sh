# A/B of the persistent traversal's waves/SIMD (PRT_OCC 7 / 8) on C4, then the GPU suite
set -o pipefail
mkdir -p gpurun_out
bash scripts/ab.sh "PRT_OCC=7" "PRT_OCC=8" "PRT_OCC=7" "PRT_OCC=8" "PRT_OCC=7" "PRT_OCC=8" || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tg.log 2>&1; rc=$?; tail -3 gpurun_out/tg.log; exit $rc
