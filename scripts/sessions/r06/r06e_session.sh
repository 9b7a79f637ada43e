set -o pipefail
bash scripts/gpu_suite.sh r06e || exit $?
for a in "1000 200" "10000 100"; do
  timeout -k 10 300 python -u scripts/tlas_drift.py $a >> gpurun_out/r06e_drift.txt 2>&1 || exit $?
done
grep instances gpurun_out/r06e_drift.txt
bash scripts/r06d_session.sh
