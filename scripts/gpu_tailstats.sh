#!/usr/bin/env bash
# Cooperative-tail counters (diagnostic build prt/ab/libprt_TS.so, -DPRT_TAIL_STATS) on the world-8 and world-1
# shares of the C4 frame: PRT_DEBUG_QUEUES=1 scripts/rank_time.py.  The in-tree library is restored afterwards.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=physically-based-ray-tracer_amd/prt
cp "$L/libprt.so" /tmp/libprt_keep.so
cp "$L/ab/libprt_TS.so" "$L/libprt.so"
PRT_DEBUG_QUEUES=1 timeout -k 10 300 python scripts/rank_time.py 8 1 > gpurun_out/tailstats.log 2>&1
rc=$?
cp /tmp/libprt_keep.so "$L/libprt.so"
grep -E "world|trace [0-9]|tail " gpurun_out/tailstats.log | tail -60
exit $rc
