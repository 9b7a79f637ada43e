# session 6: merged pipeline -- parity (merge tests, oracle full-size, golden, shard), bench merge on/off, shares, TLAS drift
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_golden_ref.py -m gpu -x -q --timeout 300 --timeout-method thread -k "merged or full_size or golden or small_all or flag or debug or progressive or ray_totals or tiles or groups" > gpurun_out/t6.log 2>&1 || { tail -40 gpurun_out/t6.log; exit 1; }
tail -2 gpurun_out/t6.log
for m in 1 0 1 0; do
  PRT_MERGE=$m timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b6_$m.log 2>&1 || { tail -20 gpurun_out/b6_$m.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('merge', sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_ms'])" gpurun_out/b6_$m.log $m
  PRT_MERGE=$m timeout -k 10 300 python scripts/rank_time.py 1 8 > gpurun_out/r6_$m.log 2>&1 || { tail -20 gpurun_out/r6_$m.log; exit 1; }
  grep world gpurun_out/r6_$m.log | sed "s/^/merge $m  /"
done
timeout -k 10 500 python scripts/tlas_drift.py 1000 200 > gpurun_out/drift6.log 2>&1 || { tail -20 gpurun_out/drift6.log; exit 1; }
grep instances gpurun_out/drift6.log | cut -c1-400
