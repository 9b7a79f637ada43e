set -o pipefail
bash scripts/gpu_suite.sh r06l || exit $?
bash scripts/gpu_prof.sh c4 r06 || exit $?
bash scripts/gpu_mem.sh c4 r06 || exit $?
for fl in default 1 4; do
  a=""; [ "$fl" != default ] && a="--inflight $fl"
  timeout -k 10 300 python3 bench.py $a > gpurun_out/r06l_bench_$fl.json 2> gpurun_out/r06l_bench_$fl.err || exit $?
  tail -1 gpurun_out/r06l_bench_$fl.json | cut -c1-200
done
