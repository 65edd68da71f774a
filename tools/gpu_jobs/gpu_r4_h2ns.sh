#!/bin/bash
# Round 4: the whole GPU suite on the refactored kernels with the default bf16x3
# split, then the NS layer with bf16x3 (default) against the f16x2 split
# (variant h2: both kernel families), interleaved; kernel stats of the default.
# Build first (here): make -C keras-geometric_amd/csrc variant NAME=h2 DEFS="-DKGX_FUSED_SPLIT=2 -DKGX_F256_SPLIT=2"
set -o pipefail
mkdir -p gpurun_out/r4h2ns
export TMPDIR=/tmp
O=gpurun_out/r4h2ns
V=keras-geometric_amd/lib/variants/libkgx_h2.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
B="--steps 20 --warmup 3 --no-cpu-baseline --no-cold"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/ns_b3_r$r.json 2>> $O/bench.err || exit $?
  KGX_LIB=$V timeout -k 10 300 python bench.py $B > $O/ns_h2_r$r.json 2>> $O/bench.err || exit $?
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/prof.log 2>&1
