# A/B: rank-0 shares with a stats read (host sync) after every frame vs none (PRT_RANK_NOSTATS=1), timers off
# (historical: the no-stats frame loop it measured is now rank_time.py's default and PRT_RANK_NOSTATS is gone; record in profiles/r03_sync_ab.txt)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/stats_ab.log
: > $out
export PRT_LAUNCH_TIMERS=0
for rep in 1 2; do
  echo "## rep $rep stats per frame" >> $out
  timeout -k 10 200 python scripts/rank_time.py 1 2 4 8 >> $out 2>&1 || exit $?
  echo "## rep $rep no stats" >> $out
  PRT_RANK_NOSTATS=1 timeout -k 10 200 python scripts/rank_time.py 1 2 4 8 >> $out 2>&1 || exit $?
done
grep -v amdgpu.ids $out
