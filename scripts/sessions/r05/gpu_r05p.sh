#!/usr/bin/env bash
# r05 final: the whole GPU suite on the final library, then the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
bash scripts/gpu_suite.sh r05p && \
timeout -k 10 400 python -u bench.py > gpurun_out/r05p_bench.log 2>&1; rc=$?
tail -2 gpurun_out/r05p_bench.log
exit $rc
