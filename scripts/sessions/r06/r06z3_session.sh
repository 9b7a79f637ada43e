set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for f in 2 3; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --inflight $f > gpurun_out/bi_${f}_${r}.json 2> gpurun_out/bi_${f}_${r}.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/bi_${f}_${r}.json').read().strip().splitlines()[-1]); print('inflight $f', round(d['value'],1), 'Mrays/s', round(d['ms_per_step'],3), 'ms')"
  done
done > gpurun_out/ab_inflight_n1.txt
cat gpurun_out/ab_inflight_n1.txt
