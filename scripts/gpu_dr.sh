set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "golden or full_size or tails or tlas or group or reference or multi" > gpurun_out/dr_tests.log 2>&1 || { tail -30 gpurun_out/dr_tests.log; exit 1; }
tail -2 gpurun_out/dr_tests.log
bash scripts/gpu_tailstats.sh | grep -E "world|trace [0-3]:|tail stats" | head -24 || exit 1
AB="BASE DR BASE DR BASE DR" RANKS="8" bash scripts/gpu_ab_libs_run.sh
