# session 9: BLAS nodes at a 128-B stride (PRT_NODE128, one line per node visit) against the packed 80-B layout:
# parity of the nd128 build (golden, full-size, query kernels), then per-kernel times interleaved (C4 bench under
# rocprofv3 kernel trace) and the world-8 share
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=physically-based-ray-tracer_amd/prt
V=${1:-nd128}
cp "$L/libprt.so" /tmp/libprt_keep.so
cp "$L/ab/libprt_$V.so" "$L/libprt.so"
timeout -k 10 600 python -u -m pytest tests/test_golden.py tests/test_golden_ref.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "golden or full_size or tails or small_all or deep or random_rays or query or occluded or intersect" > gpurun_out/s9_par.log 2>&1; rc=$?
cp /tmp/libprt_keep.so "$L/libprt.so"
tail -3 gpurun_out/s9_par.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/s9_par.log | head -20; exit $rc; }
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
kt b1 base && kt v1 $V && kt b2 base && kt v2 $V || exit 1
cp /tmp/libprt_keep.so "$L/libprt.so"
RANKS="8" bash scripts/ab_libs.sh base $V base $V
