set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06z_smoke.txt 2>&1 || { tail -5 gpurun_out/r06z_smoke.txt; exit 1; }
tail -1 gpurun_out/r06z_smoke.txt
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r06z_bench.json 2> gpurun_out/r06z_bench.err || { tail -5 gpurun_out/r06z_bench.err; exit 1; }
tail -1 gpurun_out/r06z_bench.json
