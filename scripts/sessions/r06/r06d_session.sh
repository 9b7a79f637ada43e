set -o pipefail
O=gpurun_out/r06d_ranks.txt
: > $O
for v in "PRT_RANK_INFLIGHT=4" "PRT_RANK_INFLIGHT=4 PRT_FLIGHT_GRID=4" "PRT_RANK_INFLIGHT=6" "PRT_RANK_INFLIGHT=6 PRT_FLIGHT_GRID=4" "PRT_RANK_INFLIGHT=8 PRT_FLIGHT_GRID=4" "PRT_RANK_INFLIGHT=8 PRT_FLIGHT_GRID=8" "PRT_RANK_INFLIGHT=4"; do
  echo "== $v" >> $O
  env $v timeout -k 10 240 python -u scripts/rank_time.py 4 8 >> $O 2>&1 || exit $?
done
grep -v "^  world\|RCCL version\|HIP version\|ROCm version\|Hostname\|Librccl\|amdgpu.ids\|socket.cpp" $O
