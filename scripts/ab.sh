#!/usr/bin/env bash
# A/B bench of env variants on the GPU box: scripts/ab.sh "<ENV=.. ENV=..>" "<...>" ...
# each variant: bench.py --steps 5 --warmup 1 under its own time limit; stops on any failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > "gpurun_out/ab_$i.log" 2>&1
  rc=$?
  line=$(grep '"metric"' "gpurun_out/ab_$i.log" | tail -1)
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1].ljust(36), d['value'], d['ms_per_step'], d['roofline']['launch_ms'])" "$v" "$line" 2>/dev/null || echo "$v: rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
