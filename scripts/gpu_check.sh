#!/usr/bin/env bash
# One GPU-box session: smoke -> gpu tests -> short bench (+ optional rocprof).  Each GPU step has its
# own time limit; a fault / abort / segfault / time limit (rc not in {0,1}) stops the script.
# usage: scripts/gpu_check.sh [tests|bench|prof|all] [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
what=${1:-all}
kexpr=${2:-}

step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "!! $name ended with rc=$rc: stopping (no further GPU steps)"
    exit $rc
  fi
  return 0
}

if [ "$what" = "tests" ] || [ "$what" = "all" ]; then
  step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
  if [ -n "$kexpr" ]; then
    step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$kexpr"
  else
    step pytest_gpu 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  fi
fi
if [ "$what" = "bench" ] || [ "$what" = "all" ]; then
  step bench 900 python bench.py --steps 5 --warmup 1
fi
if [ "$what" = "prof" ] || [ "$what" = "benchprof" ] || [ "$what" = "valu" ]; then
  # the machine code these passes measure (prt/codeobj.py; scripts/summarize_*.py stamp it on the summaries)
  (cd physically-based-ray-tracer_amd && python -m prt.codeobj) > gpurun_out/lib_hashes.json
fi
if [ "$what" = "prof" ] || [ "$what" = "benchprof" ]; then
  export TMPDIR=/tmp
  if [ "$what" = "benchprof" ]; then
    step bench 900 python bench.py --steps 5 --warmup 1
  fi
  step rocprof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
  step rocprof_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
  step rocprof_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
fi
if [ "$what" = "pmc" ]; then
  # scripts/gpu_check.sh pmc "<counter list>" <tag>: one extra --pmc pass (kernel-trace only, no sys/hip trace)
  export TMPDIR=/tmp
  tag=${3:-pmc}
  step "pmc_$tag" 900 rocprofv3 --pmc $kexpr --output-format csv -d "gpurun_out/pmc_$tag" -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline
fi
if [ "$what" = "valu" ] || [ "$what" = "prof" ]; then
  # VALU issue counters of the roofline (scripts/summarize_pmc.py valu): 5 SQ + 1 GRBM counters, one pass
  export TMPDIR=/tmp
  step pmc_valu 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES \
    GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_valu -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline
fi
if [ "$what" = "calib" ]; then
  # FETCH_SIZE / WRITE_SIZE against known bytes (scripts/fetch_calibration.hip; scripts/summarize_pmc.py calib)
  export TMPDIR=/tmp
  step calib_known 120 scripts/bin/fetch_calibration
  tail -n 1 gpurun_out/calib_known.log > gpurun_out/calib_known.json
  step calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_fetch -o run -- \
    scripts/bin/fetch_calibration
  step calib_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib_write -o run -- \
    scripts/bin/fetch_calibration
fi
if [ "$what" = "listpmc" ]; then
  step listpmc 300 rocprofv3 -L
fi
echo "== done"
