set -o pipefail
bash scripts/gpu_suite.sh r06x || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06x_smoke.txt 2>&1 || { tail -5 gpurun_out/r06x_smoke.txt; exit 1; }
tail -1 gpurun_out/r06x_smoke.txt
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r06x_bench.json 2> gpurun_out/r06x_bench.err || exit $?
tail -1 gpurun_out/r06x_bench.json | cut -c1-400
