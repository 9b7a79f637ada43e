#!/usr/bin/env bash
# Interleaved per-kernel A/B on one GPU box: each variant (an environment assignment list, "-" for none) runs
# bench.py one frame at a time (--inflight 1) under rocprofv3 --kernel-trace --stats, R rounds; the per-kernel mean
# durations of every run go to gpurun_out/abk_<tag>.txt (scripts/ab_kernels_summary.py).
#   scripts/ab_kernels.sh <tag> <rounds> "<variant>" ["<variant>" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1; R=$2; shift 2
mkdir -p gpurun_out
OUT=gpurun_out/abk_${T}.txt
: > "$OUT"
for r in $(seq 1 "$R"); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    envs=$v
    [ "$envs" = "-" ] && envs=""
    case "$envs" in -*) echo "bad variant '$v': assignments only (VAR=value ...), or '-'"; exit 2 ;; esac
    D=gpurun_out/abk_${T}_${r}_${i}
    rm -rf "$D"
    env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -o run -- \
      python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --inflight 1 > "$D.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$v rc=$rc" | tee -a "$OUT"; tail -5 "$D.log"; exit $rc; fi
    python3 scripts/ab_kernels_summary.py "$v" "$D" >> "$OUT" || exit 1
    tail -1 "$OUT"
  done
done
