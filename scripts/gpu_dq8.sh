# per-launch queue / wave-exit timeline (PRT_DEBUG_QUEUES) of rank 0's world-8 share, current default build
set -o pipefail
mkdir -p gpurun_out
PRT_DEBUG_QUEUES=1 timeout -k 10 300 python scripts/rank_time.py 8 > gpurun_out/dq8.log 2>&1 || { tail -20 gpurun_out/dq8.log; exit 1; }
grep -E "trace [0-9]:|iteration|world" gpurun_out/dq8.log | tail -22
