# session 10: per-kernel A/B of the shading / resolve / node-layout variants (rocprofv3 kernel trace of the C4
# bench, interleaved), the world-8 share of the candidates, then the 1,000-instance TLAS drift run
#   shpf   k_shade2 prefetches the next chunk's ray         (PRT_SHADE_PF_RAY)
#   respf  k_resmiss2 prefetches the next chunk's NEE record (PRT_RES_PF_REC)
#   dense  the resolve walks items in index order            (PRT_RES_DENSE)
#   nd128  BLAS nodes at a 128-B stride                      (PRT_NODE128)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
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
kt base1 base && kt shpf shpf && kt respf respf && kt dense1 dense && kt nd1 nd128 && kt base2 base && kt dense2 dense && kt nd2 nd128 || exit 1
cp /tmp/libprt_keep.so "$L/libprt.so"
RANKS="8" bash scripts/ab_libs.sh base dense nd128 base dense nd128 || exit 1
timeout -k 10 600 python -u scripts/tlas_drift.py 1000 200 > gpurun_out/drift10.log 2>&1; rc=$?
tail -25 gpurun_out/drift10.log
exit $rc
