#!/usr/bin/env bash
# Interleaved A/B of bench.py settings on one GPU box: each variant is an environment assignment list (or "-" for
# none) plus optional bench arguments after '::'; every variant runs once per round, R rounds.
#   scripts/ab_bench.sh <tag> <rounds> "<variant>" ["<variant>" ...]
#   e.g. scripts/ab_bench.sh hot 2 "PRT_HOT=0" "PRT_HOT=7" "PRT_HOT=7 :: --inflight 4"
# One line per run in gpurun_out/ab_<tag>.txt: variant, Mrays/s, ms/step, k_trace2 ms per launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; R=$2; shift 2
mkdir -p gpurun_out
OUT=gpurun_out/ab_${T}.txt
: > "$OUT"
for r in $(seq 1 "$R"); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    envs=$(echo ${v%%::*}); args=""  # (echo trims the blanks around the assignments)
    [[ "$v" == *"::"* ]] && args=${v#*::}
    [ "$envs" = "-" ] && envs=""
    case "$envs" in -*) echo "bad variant '$v': assignments only (VAR=value ...), or '-'"; exit 2 ;; esac
    log=gpurun_out/ab_${T}_${r}_${i}.log
    env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline $args > "$log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$v rc=$rc" | tee -a "$OUT"; tail -5 "$log"; exit $rc; fi
    python3 - "$v" "$log" >> "$OUT" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]:45s} {d['value']:9.2f} Mrays/s {d['ms_per_step']:7.3f} ms  k_trace2 {r['launch_ms']:.4f} ms "
      f"inflight {d['config']['frames_in_flight']} queues {d['config']['hw_queues']}")
EOF
    tail -1 "$OUT"
  done
done
