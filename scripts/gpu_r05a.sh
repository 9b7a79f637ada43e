#!/usr/bin/env bash
# round-5 session a: the GPU suite (+ small-builder modes), then the frames-in-flight probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_suite.sh r05a; rc=$?
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python -u scripts/inflight_probe.py 1 8 > gpurun_out/r05a_inflight.log 2>&1; rc2=$?
cat gpurun_out/r05a_inflight.log | tail -20
exit $(( rc != 0 ? rc : rc2 ))
