set -o pipefail
bash scripts/ab_bench.sh lazyb 3 "PRT_LIBPATH=physically-based-ray-tracer_amd/prt/libprt_base.so" "-" || exit $?
