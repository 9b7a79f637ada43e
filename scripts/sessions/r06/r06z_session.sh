set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=physically-based-ray-tracer_amd/prt
bash scripts/gpu_suite.sh r06zr || exit 1
bash scripts/ab_kernels.sh resdense 3 "PRT_LIBPATH=$L/libprt_before.so" "-" > /dev/null || exit 1
cat gpurun_out/abk_resdense.txt
bash scripts/ab_bench.sh resdense 3 "PRT_LIBPATH=$L/libprt_before.so" "-" || exit 1
for r in 1 2 3; do
  PRT_LIBPATH=$L/libprt_before.so PRT_TL_FRAMES=200 timeout -k 10 150 python -u scripts/share_timeline.py 8 0 2>&1 | grep '^world' | sed 's/^/before /' || exit 1
  PRT_TL_FRAMES=200 timeout -k 10 150 python -u scripts/share_timeline.py 8 0 2>&1 | grep '^world' | sed 's/^/after /' || exit 1
done > gpurun_out/ab_resdense8.txt
cat gpurun_out/ab_resdense8.txt
