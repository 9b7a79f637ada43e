# session 8: prefetch A/B (k_shade2 ray prefetch PRT_SHADE_PF_RAY, k_resmiss2 NEE-record prefetch PRT_RES_PF_REC):
# parity of the combined build, per-kernel times of each build (rocprofv3 kernel trace, C4 bench), merge 0 vs 1,
# then the 1,000-instance TLAS drift run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=physically-based-ray-tracer_amd/prt
cp "$L/libprt.so" /tmp/libprt_keep.so
cp "$L/ab/libprt_both.so" "$L/libprt.so"
timeout -k 10 600 python -u -m pytest tests/test_golden.py tests/test_golden_ref.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "golden or full_size or tails or small_all or deep or merged" > gpurun_out/s8_par.log 2>&1; rc=$?
cp /tmp/libprt_keep.so "$L/libprt.so"
tail -3 gpurun_out/s8_par.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/s8_par.log | head -20; exit $rc; }
kt() {  # kt NAME LIB MERGE
  cp "$L/ab/libprt_$2.so" "$L/libprt.so"
  rm -rf gpurun_out/kt_$1
  if [ -n "$3" ]; then export PRT_MERGE=$3; else unset PRT_MERGE; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$1 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/kt_$1.log 2>&1 || { tail -5 gpurun_out/kt_$1.log; cp /tmp/libprt_keep.so "$L/libprt.so"; exit 1; }
  echo "== $1"; grep '"metric"' gpurun_out/kt_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'])"
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows: print('%-50s calls %5s avg %10.1f us total %10.1f ms' % (r['Name'].split('(')[0][:50], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
" gpurun_out/kt_$1/run_kernel_stats.csv
}
kt base base "" && kt shpf shpf "" && kt respf respf "" && kt both both "" && kt base2 base "" && kt m1 base 1 && kt m0 base 0 || exit 1
cp /tmp/libprt_keep.so "$L/libprt.so"
timeout -k 10 600 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/drift8.log 2>&1; rc=$?
tail -25 gpurun_out/drift8.log
exit $rc
