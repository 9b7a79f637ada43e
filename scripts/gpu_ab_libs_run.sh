# library A/B (scripts/ab_libs.sh) of the variants in prt/ab/, interleaved
set -o pipefail
bash scripts/ab_libs.sh D0 L4 B64 D0 L4 B64 || exit $?
