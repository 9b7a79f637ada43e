# library A/B (scripts/ab_libs.sh) of the variants in prt/ab/, interleaved
set -o pipefail
bash scripts/ab_libs.sh A D A D A D || exit $?
