#!/usr/bin/env bash
# A/B of library builds on the GPU box: scripts/ab_libs.sh NAME...  (prt/ab/libprt_NAME.so, built beforehand)
# BENCH_ARGS overrides the bench arguments (default: C4, --steps 5 --warmup 1).  Each variant is copied over prt/libprt.so (the box's copy is scratch) and benched (C4, 5 steps) under its own
# time limit; the original library is restored at the end.  Variants run in the order given (repeat names to
# interleave).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=physically-based-ray-tracer_amd/prt
cp "$L/libprt.so" /tmp/libprt_orig.so
i=0
for v in "$@"; do
  i=$((i+1))
  cp "$L/ab/libprt_$v.so" "$L/libprt.so"
  timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 5 --warmup 1} --no-cpu-baseline > "gpurun_out/abl_$i.log" 2>&1
  rc=$?
  if [ $rc -eq 0 ] && [ -n "${RANKS:-}" ]; then  # rank 0's share of the C4 frame at these worlds (scripts/rank_time.py)
    timeout -k 10 300 python scripts/rank_time.py $RANKS > "gpurun_out/abr_$i.log" 2>&1 || rc=$?
    grep -h "world" "gpurun_out/abr_$i.log" | sed "s/^/$v  /"
  fi
  line=$(grep '"metric"' "gpurun_out/abl_$i.log" | tail -1)
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1].ljust(12), d['value'], d['ms_per_step'], d['roofline']['launch_ms'])" "$v" "$line" 2>/dev/null || echo "$v: rc=$rc"
  if [ $rc -ne 0 ]; then cp /tmp/libprt_orig.so "$L/libprt.so"; exit $rc; fi
done
cp /tmp/libprt_orig.so "$L/libprt.so"
