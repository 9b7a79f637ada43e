# kernel timelines of rank 0's world-8 share of the C4 frame, 1 and 2 batches (rocprofv3 kernel trace only)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 1 2; do
  PRT_BATCHES=$b timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt8_b$b -o run -- \
    python3 scripts/rank_time.py 8 > gpurun_out/kt8_b$b.log 2>&1 || exit $?
  tail -1 gpurun_out/kt8_b$b.log
done
