# PMC pass over the world-8 share with the streaming engine (PRT_STREAM=1) and the wavefront (PRT_STREAM=0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in 1 0; do
  PRT_STREAM=$s timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_stream$s -o run -- python3 scripts/rank_time.py 8 > gpurun_out/pmc_stream$s.log 2>&1 || { tail -5 gpurun_out/pmc_stream$s.log; exit 1; }
  grep world gpurun_out/pmc_stream$s.log
done
