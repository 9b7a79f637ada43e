# A/B: per-launch HIP event timers on (stats default) vs PRT_LAUNCH_TIMERS=0, rank-0 shares at world 1 and 8,
# interleaved, plus the 1-GPU bench line both ways; every GPU step time-limited
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/timers_ab.log
: > $out
for rep in 1 2; do
  echo "## rep $rep timers on" >> $out
  timeout -k 10 200 python scripts/rank_time.py 1 8 >> $out 2>&1 || exit $?
  echo "## rep $rep timers off" >> $out
  PRT_LAUNCH_TIMERS=0 timeout -k 10 200 python scripts/rank_time.py 1 8 >> $out 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_on.log 2>&1 || exit $?
PRT_LAUNCH_TIMERS=0 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_off.log 2>&1 || exit $?
cat $out
python - <<'PY'
import json
for f in ("on", "off"):
    d = json.loads(open(f"gpurun_out/b_{f}.log").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"].get("launch_ms"))
PY
