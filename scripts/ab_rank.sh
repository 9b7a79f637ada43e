#!/usr/bin/env bash
# A/B of env variants on the GPU box: per variant the bench line (N=1) and rank 0's share at world 8
# usage: scripts/ab_rank.sh "<ENV=.. ENV=..>" "<...>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "gpurun_out/abr_$i.log" 2>&1 || { echo "$v: bench rc=$?"; exit 1; }
  line=$(grep '"metric"' "gpurun_out/abr_$i.log" | tail -1)
  b=$(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['value'], d['ms_per_step'], d['roofline']['launch_ms'])" "$line")
  w=$(env $v timeout -k 10 300 python scripts/rank_time.py 8 4 2>&1 | grep world | awk '{printf "w%s %s ms  ", $2, $5}') || { echo "$v: rank_time failed"; exit 1; }
  echo "$v | N1 $b | $w"
done
