set -o pipefail
export TMPDIR=/tmp
for k in own side; do
  rm -rf gpurun_out/ov_$k
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ov_$k -o run -- python3 bench.py --no-cpu-baseline --context-stream $k --steps 10 > gpurun_out/ov_$k.log 2>&1 || exit $?
  tail -1 gpurun_out/ov_$k.log | cut -c1-140
  f=$(find gpurun_out/ov_$k -name "*kernel_trace.csv" | head -1)
  python3 scripts/overlap.py "$f" --last-ms 80 || exit $?
done
