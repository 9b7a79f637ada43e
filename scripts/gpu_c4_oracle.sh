# full-size C4 frame against the oracle (host cores) on the GPU box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "c4_full_size_matches_oracle" --durations=3 > gpurun_out/c4o.log 2>&1; rc=$?; tail -8 gpurun_out/c4o.log; exit $rc
