# dynamic-instance refit + BLAS builder timings, new GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dynamic or extensions or golden" > gpurun_out/tg.log 2>&1; rc=$?
tail -5 gpurun_out/tg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/dynamic_instances.py || exit $?
timeout -k 10 300 python scripts/build_time.py || exit $?
