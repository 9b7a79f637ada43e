#!/usr/bin/env bash
# One code-hash-stamped profile session of bench.py for one scene:
#   scripts/gpu_prof.sh <c4|c5> <tag>
# lib_hashes.json (the machine code measured), a --kernel-trace --stats pass, then one --pmc pass each for
# FETCH_SIZE, WRITE_SIZE, the VALU-issue counters and the stall counters (MI355X_MICROARCH.md: separate passes,
# kernel trace only).  scripts/summarize_session.py <tag> <scene> turns gpurun_out/prof_<tag>_<scene> into
# profiles/<tag>_<scene>_prof.json and profiles/current_<scene>.json (what bench.py prices).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=${1:-c4}
T=${2:-r04}
D=gpurun_out/prof_${T}_${S}
rm -rf "$D"; mkdir -p "$D"
(cd physically-based-ray-tracer_amd && python -m prt.codeobj) > "$D/lib_hashes.json" || exit 1
# one frame at a time (--inflight 1): each kernel's dispatches run alone, so their durations are the kernel's own
# (bench.py's per-launch HIP events come from its last, stats frame, which runs after the frames in flight joined)
if [ "$S" = "c5" ]; then SA="--steps 2 --warmup 1"; PA="--steps 1 --warmup 0"; else SA="--steps 5 --warmup 1"; PA="--steps 1 --warmup 1"; fi
SA="$SA --inflight 1"; PA="$PA --inflight 1"
run() {  # run <name> <limit> <rocprofv3 args...>
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" rocprofv3 "$@" --output-format csv -d "$D/$n" -o run -- python3 bench.py --scene "$S" --no-cpu-baseline $PA > "$D/$n.log" 2>&1
  local rc=$?
  echo "== $n rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$D/$n.log"; exit $rc; }
}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/stats" -o run -- \
  python3 bench.py --scene "$S" --no-cpu-baseline $SA > "$D/stats.log" 2>&1 || { tail -5 "$D/stats.log"; exit 1; }
echo "== stats ok"; tail -1 "$D/stats.log"
# the bench's own command (two frames in flight): kernel durations with the frames' overlap, for the record
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/stats_inflight" -o run -- \
  python3 bench.py --scene "$S" --no-cpu-baseline ${SA% --inflight 1} > "$D/stats_inflight.log" 2>&1 || { tail -5 "$D/stats_inflight.log"; exit 1; }
echo "== stats (frames in flight) ok"; tail -1 "$D/stats_inflight.log"
run fetch 300 --pmc FETCH_SIZE
run write 300 --pmc WRITE_SIZE
run valu 300 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
run stall 300 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS
echo "== done"
