#!/bin/bash
# Round 4: the NS fused main kernel now takes only rows of degree >= 8 and hub
# chunks (the short / tiny kernels took the rest in rounds 2-3), so the round-1
# choice of 4 gathers in flight per group is re-measured: U = 6 and U = 8 under
# a 128-VGPR cap (KGX_FUSED_MINW=4: occupancy 4 kept; U 8 spills 5) against
# the shipped U = 4, NS layer interleaved, then the tests that run the fused
# kernels under the faster variant... (A/B only; results decide).
# Build first (here): make -C keras-geometric_amd/csrc variant NAME=u6 DEFS="-DKGX_FUSED_U=6 -DKGX_FUSED_MINW=4"
#                     make -C keras-geometric_amd/csrc variant NAME=u8 DEFS="-DKGX_FUSED_U=8 -DKGX_FUSED_MINW=4"
set -o pipefail
mkdir -p gpurun_out/r4fu
export TMPDIR=/tmp
O=gpurun_out/r4fu
B="--steps 20 --warmup 3 --no-cpu-baseline --no-cold"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/ns_ship_r$r.json 2>> $O/bench.err || exit $?
  KGX_LIB=keras-geometric_amd/lib/variants/libkgx_u6.so timeout -k 10 300 python bench.py $B > $O/ns_u6_r$r.json 2>> $O/bench.err || exit $?
  KGX_LIB=keras-geometric_amd/lib/variants/libkgx_u8.so timeout -k 10 300 python bench.py $B > $O/ns_u8_r$r.json 2>> $O/bench.err || exit $?
done
for v in u6 u8; do
  KGX_LIB=keras-geometric_amd/lib/variants/libkgx_$v.so timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/prof_$v -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/prof_$v.log 2>&1 || exit $?
done
