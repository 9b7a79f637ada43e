# session 13: the full GPU suite on the new defaults (shading kernel ray prefetch, dense resolve, sync-free
# single-workgroup instance-BVH rebuild), the 1,000-instance drift (refit only / trigger / every frame), and the
# per-wave append A/B (PRT_WAVE_APPEND) under the kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s13_tests.log 2>&1; rc=$?
tail -5 gpurun_out/s13_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/s13_tests.log | head -30; exit $rc; }
timeout -k 10 280 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/drift13.log 2>&1 || { tail -5 gpurun_out/drift13.log; exit 1; }
grep instances gpurun_out/drift13.log
L=physically-based-ray-tracer_amd/prt
cp "$L/libprt.so" /tmp/libprt_keep.so
kt() {  # kt NAME LIB
  cp "$L/ab/libprt_$2.so" "$L/libprt.so"
  rm -rf gpurun_out/kt_$1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$1 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/kt_$1.log 2>&1 || { tail -5 gpurun_out/kt_$1.log; cp /tmp/libprt_keep.so "$L/libprt.so"; exit 1; }
  echo "== $1"; grep '"metric"' gpurun_out/kt_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'])"
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:4]: print('%-50s calls %5s avg %10.1f us total %10.1f ms' % (r['Name'].split('(')[0][:50], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
" gpurun_out/kt_$1/run_kernel_stats.csv
}
kt base1 base && kt wapp1 wapp && kt base2 base && kt wapp2 wapp || exit 1
cp /tmp/libprt_keep.so "$L/libprt.so"
RANKS="8" bash scripts/ab_libs.sh base wapp base wapp
