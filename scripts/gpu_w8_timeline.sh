# kernel-by-kernel timeline of one world-8 rank-0 share (rocprofv3 kernel trace), ABI-7 frame loop without timers
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/w8 -o run -- python3 scripts/rank_time.py 8 > gpurun_out/w8.log 2>&1 || { tail -20 gpurun_out/w8.log; exit 1; }
f=$(find gpurun_out/w8 -name '*kernel_trace.csv' | head -1)
python3 scripts/frame_timeline.py "$f" > gpurun_out/w8_timeline.txt && cat gpurun_out/w8_timeline.txt
