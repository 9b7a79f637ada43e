set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_inflight.py tests/test_brdf_vectors.py tests/test_gpu_shard.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06c_gpu.log 2>&1; rc=$?; tail -8 gpurun_out/r06c_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
for v in "PRT_RANK_INFLIGHT=2" "PRT_RANK_INFLIGHT=4" "PRT_RANK_INFLIGHT=4 GPU_MAX_HW_QUEUES=8" "PRT_RANK_INFLIGHT=4 PRT_FLIGHT_PRIO=high"; do
  echo "== $v" >> gpurun_out/r06c_ranks.txt
  env $v timeout -k 10 240 python -u scripts/rank_time.py >> gpurun_out/r06c_ranks.txt 2>&1 || exit $?
done
grep -v "^  world" gpurun_out/r06c_ranks.txt
