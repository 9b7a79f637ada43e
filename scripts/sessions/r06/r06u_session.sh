set -o pipefail
timeout -k 10 300 python -u scripts/rank_time.py > gpurun_out/r06u_ranks_c4.txt 2>&1 || exit $?
grep -v "RCCL version\|HIP version\|ROCm version\|Hostname\|Librccl\|amdgpu.ids\|socket.cpp\|^  world" gpurun_out/r06u_ranks_c4.txt
PRT_RANK_STREAM=side timeout -k 10 300 python -u scripts/rank_time.py 8 > gpurun_out/r06u_ranks_c4_side.txt 2>&1 || exit $?
grep -v "RCCL version\|HIP version\|ROCm version\|Hostname\|Librccl\|amdgpu.ids\|socket.cpp\|^  world" gpurun_out/r06u_ranks_c4_side.txt
timeout -k 10 400 python -u scripts/rank_time.py c5 > gpurun_out/r06u_ranks_c5.txt 2>&1 || exit $?
grep -v "RCCL version\|HIP version\|ROCm version\|Hostname\|Librccl\|amdgpu.ids\|socket.cpp\|^  world" gpurun_out/r06u_ranks_c5.txt
: > gpurun_out/r06u_drift.txt
for a in "1000 200" "10000 100"; do
  PRT_DRIFT_STREAM=own PRT_DRIFT_INFLIGHT=2 timeout -k 10 300 python -u scripts/tlas_drift.py $a >> gpurun_out/r06u_drift.txt 2>&1 || exit $?
done
grep instances gpurun_out/r06u_drift.txt
