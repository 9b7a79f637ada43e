# re-check of traversal knobs at the current default (7 waves): refill threshold 32 / 48
set -o pipefail
mkdir -p gpurun_out
bash scripts/ab.sh "PRT_TRAV=refill32" "PRT_TRAV=refill48" "PRT_TRAV=refill32" "PRT_TRAV=refill48" "PRT_TRAV=refill32" "PRT_TRAV=refill48" || exit $?
for v in "PRT_TRAV=refill32" "PRT_TRAV=refill48"; do echo "$v"; env $v timeout -k 10 300 python scripts/rank_time.py 8 || exit $?; done
