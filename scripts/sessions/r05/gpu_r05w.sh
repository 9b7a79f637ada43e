#!/usr/bin/env bash
# round-5 session w: the resolve kernels load the ending paths' stack records and s1 up front (A: this tree; B:
# ab/B, built with -DPRT_RES_AHEAD=0); the whole GPU suite on A, then interleaved bench / world-8 share A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
T=${1:-r05w}
bash scripts/gpu_suite.sh $T || exit $?
bench() {  # bench <tag> <dir>
  timeout -k 10 300 python $2/bench.py --warmup 3 --steps 30 --no-cpu-baseline > gpurun_out/${T}_$1.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_ms'])" gpurun_out/${T}_$1.log $1
}
for k in 1 2 3; do
  bench A_$k .
  bench B_$k ab/B
done
for k in 1 2; do
  for v in A B; do
    d=.; [ $v = B ] && d=ab/B
    GPU_MAX_HW_QUEUES=8 PRT_RANK_INFLIGHT=4 timeout -k 10 300 python -u $d/scripts/rank_time.py 1 8 > gpurun_out/${T}_rank_${v}_$k.log 2>&1 || exit $?
    echo "rank $v"; tail -2 gpurun_out/${T}_rank_${v}_$k.log
  done
done
