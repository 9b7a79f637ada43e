# session 7: per-kernel times of the merged vs unmerged pipeline (rocprofv3 kernel trace, C4 bench)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1 0; do
  rm -rf gpurun_out/kt_m$m
  PRT_MERGE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_m$m -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/kt_m$m.log 2>&1 || { tail -5 gpurun_out/kt_m$m.log; exit 1; }
  echo "== merge $m"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows: print('%-50s calls %5s avg %10.1f us total %10.1f ms' % (r['Name'].split('(')[0][:50], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
" gpurun_out/kt_m$m/run_kernel_stats.csv
done
