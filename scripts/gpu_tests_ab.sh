#!/usr/bin/env bash
# GPU suite on the in-tree library, then a library A/B (scripts/gpu_ab_libs_run.sh; AB / RANKS from the env)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_ab_libs_run.sh
