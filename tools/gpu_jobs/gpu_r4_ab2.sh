#!/bin/bash
# Round 4, same-box A/B (interleaved, two rounds): NS GCN layer, shipped
# library (fused main kernel U = 4, PF = 4 at F_in 128) vs libkgx_u8pf2.so
# (U = 8 gathers in flight, 2-row prefetch, every instantiation); C5 SAGEConv
# mean: fused update (narrow main kernel U = 8, PF = 2) vs KGX_TINY_ACC_EARLY=1
# (libkgx_accearly.so) vs the two-step path (KGX_FUSED_SAGE=0); kernel stats of
# the fused C5 layer.
# Build first (here): make -C keras-geometric_amd/csrc variant NAME=accearly DEFS=-DKGX_TINY_ACC_EARLY=1 and
#   variant NAME=u8pf2 DEFS="-DKGX_FUSED_U=8 -DKGX_FUSED_PF=2"
set -o pipefail
mkdir -p gpurun_out/r4ab2
export TMPDIR=/tmp
V=keras-geometric_amd/lib/variants
B="--no-cpu-baseline --no-cold"
O=gpurun_out/r4ab2
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 $B > $O/ns_r$r.json 2>> $O/bench.err || exit $?
  KGX_LIB=$V/libkgx_u8pf2.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 $B > $O/ns_u8pf2_r$r.json 2>> $O/bench.err || exit $?
  timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 $B > $O/fused_r$r.json 2>> $O/bench.err || exit $?
  KGX_LIB=$V/libkgx_accearly.so timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 $B \
    > $O/accearly_r$r.json 2>> $O/bench.err || exit $?
  KGX_FUSED_SAGE=0 timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 $B > $O/twostep_r$r.json 2>> $O/bench.err || exit $?
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python3 bench.py --config c5 --steps 10 --warmup 2 $B > $O/prof.log 2>&1
