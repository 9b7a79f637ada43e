set -o pipefail
bash scripts/gpu_suite.sh r06j || exit $?
: > gpurun_out/r06j_drift.txt
for fl in 1 2; do
  for a in "1000 200" "10000 100"; do
    PRT_DRIFT_INFLIGHT=$fl timeout -k 10 300 python -u scripts/tlas_drift.py $a >> gpurun_out/r06j_drift.txt 2>&1 || exit $?
  done
done
grep instances gpurun_out/r06j_drift.txt
bash scripts/gpu_prof.sh c4 r06 || exit $?
bash scripts/gpu_mem.sh c4 r06 || exit $?
