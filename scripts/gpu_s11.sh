# session 11: parity of the combined shading build (all3 = hit/miss partition PRT_SHADE_SORT + ray prefetch
# PRT_SHADE_PF_RAY + dense resolve PRT_RES_DENSE), then per-kernel times interleaved against base, sort alone and
# pfd (prefetch + dense), and the world-8 share
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=physically-based-ray-tracer_amd/prt
cp "$L/libprt.so" /tmp/libprt_keep.so
cp "$L/ab/libprt_all3.so" "$L/libprt.so"
timeout -k 10 700 python -u -m pytest tests/test_golden.py tests/test_golden_ref.py tests/test_gpu_parity.py tests/test_extensions.py -m gpu -x -q --timeout 300 --timeout-method thread -k "golden or full_size or tails or small_all or deep or merged or mode or flag or progressive or extension or c5" > gpurun_out/s11_par.log 2>&1; rc=$?
cp /tmp/libprt_keep.so "$L/libprt.so"
tail -3 gpurun_out/s11_par.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/s11_par.log | head -20; exit $rc; }
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
kt base1 base && kt sort1 sort && kt all1 all3 && kt pfd1 pfd && kt base2 base && kt sort2 sort && kt all2 all3 && kt pfd2 pfd || exit 1
cp /tmp/libprt_keep.so "$L/libprt.so"
RANKS="8" bash scripts/ab_libs.sh base all3 base all3
