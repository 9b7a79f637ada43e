#!/usr/bin/env bash
# library A/B on C4 ($AB4) and on C5 ($AB5) (scripts/ab_libs.sh), one GPU session
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/ab_libs.sh ${AB4} || exit $?
BENCH_ARGS="--scene c5 --steps 3 --warmup 1" bash scripts/ab_libs.sh ${AB5}
