set -o pipefail
mkdir -p gpurun_out
for occ in 7 6 5 4 7; do
  echo "== PRT_OCC=$occ"
  PRT_OCC=$occ timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/occ$occ.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/occ$occ.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['launch_ms'])"
  PRT_OCC=$occ timeout -k 10 200 python scripts/rank_time.py 1 8 > gpurun_out/rank_occ$occ.log 2>&1 || exit $?
  cat gpurun_out/rank_occ$occ.log | grep world
done
