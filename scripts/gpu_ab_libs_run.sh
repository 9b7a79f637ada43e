# library A/B (scripts/ab_libs.sh) of the variants in prt/ab/, interleaved; then the full-size parity of the
# variant named in $PARITY (copied over prt/libprt.so for that pytest run only)
set -o pipefail
bash scripts/ab_libs.sh ${AB:-D0 FP OV FO D0 FP OV FO} || exit $?
if [ -n "${PARITY:-}" ]; then
  L=physically-based-ray-tracer_amd/prt
  cp "$L/libprt.so" /tmp/libprt_keep.so
  cp "$L/ab/libprt_$PARITY.so" "$L/libprt.so"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "${PARITY_K:-full_size or golden or reference}" > gpurun_out/ab_parity.log 2>&1; rc=$?
  cp /tmp/libprt_keep.so "$L/libprt.so"
  tail -5 gpurun_out/ab_parity.log
  exit $rc
fi
