#!/usr/bin/env bash
# PLOC search radius A/B: scripts/build_time.py only-ploc on C4 and the Spaceship for each prt/ab/libprt_R*.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=physically-based-ray-tracer_amd/prt
cp "$L/libprt.so" /tmp/libprt_keep.so
rc=0
for v in ${VARIANTS:-R16 R32 R64}; do
  cp "$L/ab/libprt_$v.so" "$L/libprt.so"
  for s in c4 ship; do
    timeout -k 10 300 python scripts/build_time.py only-ploc $s > "gpurun_out/ploc_${v}_$s.log" 2>&1 || { rc=$?; break 2; }
    echo "$v $s: $(grep PLOC gpurun_out/ploc_${v}_$s.log)"
  done
done
cp /tmp/libprt_keep.so "$L/libprt.so"
exit $rc
