# session 2: bench lines priced by the r04a profiles (C4, C5), instance-BVH drift with the node-area trigger
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || { tail -20 gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log | cut -c1-1500
timeout -k 10 300 python bench.py --scene c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || { tail -20 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log | cut -c1-1500
timeout -k 10 500 python scripts/tlas_drift.py 1000 200 > gpurun_out/drift.log 2>&1 || { tail -20 gpurun_out/drift.log; exit 1; }
cat gpurun_out/drift.log
