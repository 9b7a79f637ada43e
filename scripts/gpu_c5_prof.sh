#!/usr/bin/env bash
# C5 (3840x2160, 16 spp, depth 8, area light MIS) on one GPU: bench line, rocprofv3 kernel stats and the HBM /
# VALU PMC passes of its traversal kernel; plus rank 0's share of the C4 frame at world 1/2/4/8
# (scripts/rank_time.py).  Each GPU step under its own limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 6 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step rank_time 300 python scripts/rank_time.py
step c5_bench 300 python bench.py --scene c5 --steps 3 --warmup 1 --no-cpu-baseline
step c5_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5_stats -o run -- \
  python3 bench.py --scene c5 --steps 2 --warmup 1 --no-cpu-baseline
step c5_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c5_fetch -o run -- \
  python3 bench.py --scene c5 --steps 1 --warmup 1 --no-cpu-baseline
step c5_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/c5_write -o run -- \
  python3 bench.py --scene c5 --steps 1 --warmup 1 --no-cpu-baseline
step c5_valu 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/c5_valu -o run -- python3 bench.py --scene c5 --steps 1 --warmup 1 --no-cpu-baseline
echo "== done"
