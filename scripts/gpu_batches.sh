# wavefront batches A/B: parity tests, bench per batch count, rank-0 share per world size, world-8 kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "batches or pipelines or tiles" > gpurun_out/t2.log 2>&1; rc=$?; tail -3 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab.sh "PRT_BATCHES=1" "PRT_BATCHES=2" "PRT_BATCHES=3" || exit $?
for b in 1 2 3; do echo "batches $b"; PRT_BATCHES=$b timeout -k 10 300 python scripts/rank_time.py 1 2 4 8 || exit $?; done
PRT_BATCHES=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt8_b2 -o run -- \
    python3 scripts/rank_time.py 8 > gpurun_out/kt8_b2.log 2>&1 || exit $?
