# A/B: wavefront batches on concurrent streams with a shrunk persistent trace grid (PRT_BATCHES, PRT_TRACE_WAVES):
# C4 bench at N = 1, then rank 0's share at world 8 (scripts/rank_time.py)
set -o pipefail
mkdir -p gpurun_out
bash scripts/ab.sh "PRT_BATCHES=1" "PRT_BATCHES=2" "PRT_BATCHES=2 PRT_TRACE_WAVES=4" "PRT_BATCHES=2 PRT_TRACE_WAVES=3" "PRT_BATCHES=1 PRT_TRACE_WAVES=5" || exit $?
for v in "PRT_BATCHES=1" "PRT_BATCHES=2 PRT_TRACE_WAVES=4" "PRT_BATCHES=2 PRT_TRACE_WAVES=3" "PRT_BATCHES=3 PRT_TRACE_WAVES=3" "PRT_BATCHES=2 PRT_TRACE_WAVES=5"; do echo "$v"; env $v PRT_BATCH_MIN=16384 timeout -k 10 300 python scripts/rank_time.py 8 || exit $?; done
