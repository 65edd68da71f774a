mkdir -p gpurun_out
for d in 0 1 2 3; do echo "debug=$d"; KGX_LIB=keras-geometric_amd/lib/variants/libkgx_dexp.so KGX_DENSE_DEBUG=$d timeout -k 10 120 python tools/bench_dense.py --only NS,C4 --reps 10 || exit 1; done
