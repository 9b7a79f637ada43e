#!/usr/bin/env bash
# round-5 session g: session f (build phases per radius, drift, hardware queues) + code-hash-stamped profiles of C4
# and C5 (scripts/gpu_prof.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
bash scripts/gpu_prof.sh c4 r05 || exit $?
bash scripts/gpu_prof.sh c5 r05 || exit $?
bash scripts/gpu_r05f.sh r05g || exit $?
