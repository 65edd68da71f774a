# kgx_dense cost decomposition (experiment build, KGX_DENSE_DEBUG bits: 1 no MFMA, 2 no stores, 4 no loads/split)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/dexp.log
for d in ${DBG:-0 1 2 4 6 3}; do echo "debug=$d" >> gpurun_out/dexp.log; KGX_LIB=keras-geometric_amd/lib/variants/libkgx_dexp.so KGX_DENSE_DEBUG=$d timeout -k 10 120 python tools/bench_dense.py --only ${ONLY:-NS,C4} --reps 10 >> gpurun_out/dexp.log 2>&1 || exit 1; done
