set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for w in 8 4; do
    n=$((w == 8 ? 200 : 100))
    PRT_TL_FRAMES=$n timeout -k 10 150 python -u scripts/share_timeline.py $w 0 2>&1 | grep '^world' | sed 's/^/merged   /' || exit 1
    PRT_MERGE=0 PRT_TL_FRAMES=$n timeout -k 10 150 python -u scripts/share_timeline.py $w 0 2>&1 | grep '^world' | sed 's/^/unmerged /' || exit 1
  done
done > gpurun_out/ab_merge_third.txt
cat gpurun_out/ab_merge_third.txt
