set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_inflight.py tests/test_gpu_parity.py -q -k "tlas or inflight or instance or materials" --timeout 120 --timeout-method thread > gpurun_out/r06n_tests.log 2>&1 || { tail -30 gpurun_out/r06n_tests.log; exit 1; }
tail -2 gpurun_out/r06n_tests.log
: > gpurun_out/r06n_drift.txt
for fl in 1 2; do
  for a in "1000 200" "10000 100"; do
    PRT_DRIFT_INFLIGHT=$fl timeout -k 10 300 python -u scripts/tlas_drift.py $a >> gpurun_out/r06n_drift.txt 2>&1 || exit $?
  done
done
grep instances gpurun_out/r06n_drift.txt
timeout -k 10 400 python3 bench.py --scene c5 --steps 4 --warmup 1 > gpurun_out/r06n_c5_bench.json 2> gpurun_out/r06n_c5_bench.err || exit $?
tail -1 gpurun_out/r06n_c5_bench.json | cut -c1-200
