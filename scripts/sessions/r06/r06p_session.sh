set -o pipefail
bash scripts/gpu_suite.sh r06p || exit $?
timeout -k 10 240 python -u scripts/inst_update_probe.py 10000 > gpurun_out/r06p_probe.txt 2>&1 || exit $?
grep N= gpurun_out/r06p_probe.txt
: > gpurun_out/r06p_drift.txt
for fl in 1 2; do
  for a in "1000 200" "10000 100"; do
    PRT_DRIFT_INFLIGHT=$fl timeout -k 10 300 python -u scripts/tlas_drift.py $a >> gpurun_out/r06p_drift.txt 2>&1 || exit $?
  done
done
grep instances gpurun_out/r06p_drift.txt
timeout -k 10 300 python -u scripts/rank_time.py > gpurun_out/r06p_ranks_c4.txt 2>&1 || exit $?
grep -v "RCCL version\|HIP version\|ROCm version\|Hostname\|Librccl\|amdgpu.ids\|socket.cpp\|^  world" gpurun_out/r06p_ranks_c4.txt
timeout -k 10 400 python -u scripts/rank_time.py c5 > gpurun_out/r06p_ranks_c5.txt 2>&1 || exit $?
grep -v "RCCL version\|HIP version\|ROCm version\|Hostname\|Librccl\|amdgpu.ids\|socket.cpp\|^  world" gpurun_out/r06p_ranks_c5.txt
