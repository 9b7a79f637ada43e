# A/B of the traversal tails (PRT_TAIL 0 none / 1 cooperative / 2 group / 3 both): C4 bench + rank-0 share at world 8
set -o pipefail
mkdir -p gpurun_out
bash scripts/ab.sh "PRT_TAIL=1" "PRT_TAIL=2" "PRT_TAIL=3" "PRT_TAIL=0" || exit $?
for m in 1 2 3; do echo "tail $m"; PRT_TAIL=$m timeout -k 10 300 python scripts/rank_time.py 1 8 || exit $?; done
