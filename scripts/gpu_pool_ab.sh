# triangle-pool A/B (prt_persist.h POOL): parity of the pool build on the golden / full-size tests, then
# interleaved benches and rank-0 shares of base / pool builds (scripts/ab_libs.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=physically-based-ray-tracer_amd/prt
cp "$L/libprt.so" /tmp/libprt_keep.so
cp "$L/ab/libprt_${1:-pool88}.so" "$L/libprt.so"
timeout -k 10 900 python -u -m pytest tests/test_golden.py tests/test_golden_ref.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "golden or full_size or tails or random_rays or small_all or tiles or deep or tlas or many" > gpurun_out/tpool.log 2>&1; rc=$?
cp /tmp/libprt_keep.so "$L/libprt.so"
tail -3 gpurun_out/tpool.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/tpool.log | head -20; exit $rc; }
RANKS="1 8" bash scripts/ab_libs.sh base ${1:-pool88} base ${1:-pool88} ${2:-}
