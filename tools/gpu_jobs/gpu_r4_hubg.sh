#!/bin/bash
# Round 4: EXACT hub rows in 4 column groups of 32 features (KGX_HUB_G=8,
# lib/variants/libkgx_hubg8.so) against 2 groups of 64 (shipped), NS --exact,
# interleaved; the bit-identity tests under the variant.
# Build first (here): make -C keras-geometric_amd/csrc variant NAME=hubg8 DEFS=-DKGX_HUB_G=8
set -o pipefail
mkdir -p gpurun_out/r4h
export TMPDIR=/tmp
O=gpurun_out/r4h
V=keras-geometric_amd/lib/variants/libkgx_hubg8.so
KGX_LIB=$V timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "exact or bitwise or bit_identical" \
  --timeout 240 --timeout-method thread > $O/pytest_exact_hubg8.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_exact_hubg8.log
[ $rc -eq 0 ] || exit $rc
B="--exact --steps 20 --warmup 3 --no-cpu-baseline --no-cold"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/exact_g16_r$r.json 2>> $O/bench.err || exit $?
  KGX_LIB=$V timeout -k 10 300 python bench.py $B > $O/exact_g8_r$r.json 2>> $O/bench.err || exit $?
done
KGX_LIB=$V timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python3 bench.py $B > $O/prof.log 2>&1
