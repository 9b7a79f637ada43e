set -o pipefail
export TMPDIR=/tmp
for v in "4 own rccl" "4 side rccl" "2 own plain" "4 own plain"; do
  t=$(echo $v | tr ' ' '_')
  rm -rf gpurun_out/qp_$t
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/qp_$t -o run -- python3 scripts/queue_probe.py $v > gpurun_out/qp_$t.log 2>&1 || exit $?
  grep "in flight" gpurun_out/qp_$t.log
  f=$(find gpurun_out/qp_$t -name "*kernel_trace.csv" | head -1)
  python3 scripts/overlap.py "$f" --last-ms 60 || exit $?
done
