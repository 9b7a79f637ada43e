# library A/B (scripts/ab_libs.sh) of the variants in prt/ab/, interleaved
set -o pipefail
bash scripts/ab_libs.sh S4 S5 S6 S4 S5 S6 || exit $?
