set -o pipefail
: > gpurun_out/r06w_cumask.txt
for r in 1 2; do
  for m in 0 1; do
    echo "== PRT_FLIGHT_CUMASK=$m round $r" >> gpurun_out/r06w_cumask.txt
    if [ $m = 1 ]; then export PRT_FLIGHT_CUMASK=1; else unset PRT_FLIGHT_CUMASK; fi
    timeout -k 10 200 python -u scripts/rank_time.py 8 >> gpurun_out/r06w_cumask.txt 2>&1 || exit $?
  done
done
unset PRT_FLIGHT_CUMASK
grep "==\|c4 world" gpurun_out/r06w_cumask.txt
