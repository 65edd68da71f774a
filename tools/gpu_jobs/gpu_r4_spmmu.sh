#!/bin/bash
# Round 4: C5 SAGE-mean layer, spmm_kernel with 8 gathers in flight per group
# (KGX_SPMM_U=8: 64 VGPRs unweighted, occupancy 8 kept) against 6, interleaved.
# Build first (here): make -C keras-geometric_amd/csrc variant NAME=u8 DEFS=-DKGX_SPMM_U=8
set -o pipefail
mkdir -p gpurun_out/r4u
export TMPDIR=/tmp
O=gpurun_out/r4u
V=keras-geometric_amd/lib/variants/libkgx_u8.so
B="--config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-cold"
for r in 1 2 3; do
  timeout -k 10 300 python bench.py $B > $O/c5_u6_r$r.json 2>> $O/bench.err || exit $?
  KGX_LIB=$V timeout -k 10 300 python bench.py $B > $O/c5_u8_r$r.json 2>> $O/bench.err || exit $?
done
