# A/B: k_trace2 rays-per-wave cap for launches with fewer rays than lanes (PRT_TRACE_CAP_MIN; 0 = off),
# rank-0 shares at world 1 / 4 / 8, interleaved; every GPU step time-limited
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/cap_ab.log
: > $out
for rep in 1 2; do
  for cap in 0 1 4 16; do
    echo "## rep $rep cap_min $cap" >> $out
    PRT_TRACE_CAP_MIN=$cap timeout -k 10 200 python scripts/rank_time.py 1 4 8 >> $out 2>&1 || { cat $out; exit 1; }
  done
done
grep -v amdgpu.ids $out
