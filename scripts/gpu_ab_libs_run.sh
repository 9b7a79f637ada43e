# library A/B (scripts/ab_libs.sh) of the variants in prt/ab/, interleaved, on C5 at reduced steps
set -o pipefail
BENCH_ARGS="--scene c5 --steps 3 --warmup 1" bash scripts/ab_libs.sh E2 E3 E2 E3 || exit $?
