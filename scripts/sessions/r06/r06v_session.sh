set -o pipefail
export TMPDIR=/tmp
for m in 0 1; do
  for v in "4 own plain" "2 own plain" "4 own rccl"; do
    t=$(echo $v | tr ' ' '_')_m$m
    rm -rf gpurun_out/qv_$t
    if [ $m = 1 ]; then export PRT_FLIGHT_CUMASK=1; else unset PRT_FLIGHT_CUMASK; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/qv_$t -o run -- python3 scripts/queue_probe.py $v > gpurun_out/qv_$t.log 2>&1 || exit $?
    echo "cumask=$m $(grep 'in flight' gpurun_out/qv_$t.log)"
    f=$(find gpurun_out/qv_$t -name "*kernel_trace.csv" | head -1)
    python3 scripts/overlap.py "$f" --last-ms 60 | grep "span\|queue" || exit $?
  done
done
unset PRT_FLIGHT_CUMASK
bash scripts/ab_bench.sh cumask 2 "-" "PRT_FLIGHT_CUMASK=1" "- :: --inflight 4" "PRT_FLIGHT_CUMASK=1 :: --inflight 4" || exit $?
