# lane-usage histogram of k_trace2 (diagnostic build prt/ab/libprt_lanestats.so, scripts/lane_stats.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=physically-based-ray-tracer_amd/prt
cp "$L/libprt.so" /tmp/libprt_orig.so
cp "$L/ab/libprt_lanestats.so" "$L/libprt.so"
timeout -k 10 400 python scripts/lane_stats.py ${1:-r04} > gpurun_out/lanestats.log 2>&1; rc=$?
cp /tmp/libprt_orig.so "$L/libprt.so"
cat gpurun_out/lanestats.log | tail -5
mkdir -p gpurun_out/profiles && cp profiles/${1:-r04}_lane_stats.json gpurun_out/profiles/ 2>/dev/null
exit $rc
