set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  PRT_TL_FRAMES=200 timeout -k 10 150 python -u scripts/share_timeline.py 8 0 2>&1 | grep '^world' | sed 's/^/tail on  /' || exit 1
  PRT_TAIL=0 PRT_TL_FRAMES=200 timeout -k 10 150 python -u scripts/share_timeline.py 8 0 2>&1 | grep '^world' | sed 's/^/tail off /' || exit 1
done > gpurun_out/ab_tail8.txt
cat gpurun_out/ab_tail8.txt
