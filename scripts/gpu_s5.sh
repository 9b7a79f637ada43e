# session 5: device TLAS tree quality by PLOC radius; pool A/B with partial passes only when <= 8 lanes have node work
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TLAS_MODES=radius timeout -k 10 600 python scripts/tlas_drift.py 1000 60 > gpurun_out/drift_radius.log 2>&1 || { tail -20 gpurun_out/drift_radius.log; exit 1; }
cat gpurun_out/drift_radius.log
RANKS="1 8" bash scripts/ab_libs.sh base pool88p8 pool88p0 base pool88p8 pool88p0
