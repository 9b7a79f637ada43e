set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_inflight.py -q --timeout 240 --timeout-method thread > gpurun_out/r06r_tests.log 2>&1 || { tail -30 gpurun_out/r06r_tests.log; exit 1; }
tail -2 gpurun_out/r06r_tests.log
for r in 1 2; do
  timeout -k 10 300 python3 bench.py > gpurun_out/r06r_bench_$r.json 2> gpurun_out/r06r_bench_$r.err || exit $?
  tail -1 gpurun_out/r06r_bench_$r.json | cut -c1-160
done
timeout -k 10 300 python3 bench.py --inflight 4 > gpurun_out/r06r_bench_fl4.json 2> gpurun_out/r06r_bench_fl4.err || exit $?
tail -1 gpurun_out/r06r_bench_fl4.json | cut -c1-160
timeout -k 10 300 python -u scripts/rank_time.py > gpurun_out/r06r_ranks_c4.txt 2>&1 || exit $?
grep -v "RCCL version\|HIP version\|ROCm version\|Hostname\|Librccl\|amdgpu.ids\|socket.cpp\|^  world" gpurun_out/r06r_ranks_c4.txt
