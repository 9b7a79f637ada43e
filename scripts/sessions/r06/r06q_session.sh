set -o pipefail
: > gpurun_out/r06q_stream_ab.txt
for r in 1 2; do
  for k in own side; do
    echo "== PRT_RANK_STREAM=$k round $r" >> gpurun_out/r06q_stream_ab.txt
    PRT_RANK_STREAM=$k timeout -k 10 200 python -u scripts/rank_time.py 8 4 >> gpurun_out/r06q_stream_ab.txt 2>&1 || exit $?
  done
done
grep "==\|c4 world" gpurun_out/r06q_stream_ab.txt
