#!/usr/bin/env bash
# round-5 session a: the GPU suite (+ small-builder modes), then the frames-in-flight probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
bash scripts/gpu_suite.sh r05a; rc=$?
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python -u scripts/inflight_probe.py 1 8 > gpurun_out/r05a_inflight.log 2>&1; rc2=$?
cat gpurun_out/r05a_inflight.log | tail -20
[ $rc2 -eq 0 ] || exit $rc2
# traversal occupancy A/B (7 vs 8 waves/SIMD; C4's BLAS is 9 levels deep, so the 8-group LDS stack holds it)
for r in 1 2; do for o in 7 8; do
  PRT_OCC=$o timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r05a_occ${o}_$r.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_ms'])" gpurun_out/r05a_occ${o}_$r.log occ$o
done; done
exit $rc
