#!/usr/bin/env bash
# Memory-pipeline counters of one bench.py scene: which stage of the vector-memory path bounds
# the traversal kernel.  One --pmc pass per block group (MI355X_MICROARCH.md: <= 2 TA, 2 TD, 4 TCP, 4 TCC, 2 GRBM
# per pass), each under its own time limit; the library's code hashes first, so the summary is tied to the build.
#   scripts/gpu_mem.sh <c4|c5> <tag>      -> gpurun_out/mem_<tag>_<scene>/<pass>/run_counter_collection.csv
# scripts/summarize_mem.py <tag> <scene> turns the session into profiles/<tag>_<scene>_mem.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=${1:-c4}
T=${2:-r06}
D=gpurun_out/mem_${T}_${S}
rm -rf "$D"; mkdir -p "$D"
(cd physically-based-ray-tracer_amd && python -m prt.codeobj) > "$D/lib_hashes.json" || exit 1
timeout -s KILL 60 rocprofv3 --list-avail > "$D/avail.txt" 2>&1
echo "== avail rc=$?"
PA="--steps 1 --warmup 1 --inflight 1"
[ "$S" = "c5" ] && PA="--steps 1 --warmup 0 --inflight 1"
run() {  # run <name> <counters...>; a refused counter set (rc 1) is logged and skipped, a kill ends the session
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$D/$n" -o run -- \
    python3 bench.py --scene "$S" --no-cpu-baseline $PA > "$D/$n.log" 2>&1
  local rc=$?
  echo "== $n rc=$rc"
  case $rc in 0) ;; 124|137|134|139) tail -5 "$D/$n.log"; exit $rc ;; *) tail -3 "$D/$n.log" ;; esac
}
run ta TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT
run ta2 TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
run td TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
run tcp TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
run tcp2 TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_GATE_EN1_sum GRBM_GUI_ACTIVE
run tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE
run sq SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE
echo "== done"
