#!/bin/bash
# Round 4: EXACT mode with the degree <= 7 suffix of the degree-ordered rows on
# spmm_short_kernel (kgx_spmm_ex's n_long_items with items = NULL): every
# EXACT / bit-identity GPU test, then an interleaved A/B against
# KGX_SHORT_ROWS=0 (the whole row list on spmm_kernel, as before), NS --exact.
set -o pipefail
mkdir -p gpurun_out/r4e
export TMPDIR=/tmp
O=gpurun_out/r4e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "exact or bitwise or bit_identical" \
  --timeout 240 --timeout-method thread > $O/pytest_exact.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_exact.log
[ $rc -eq 0 ] || exit $rc
B="--exact --steps 20 --warmup 3 --no-cpu-baseline --no-cold"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/exact_short_r$r.json 2>> $O/bench.err || exit $?
  KGX_SHORT_ROWS=0 timeout -k 10 300 python bench.py $B > $O/exact_noshort_r$r.json 2>> $O/bench.err || exit $?
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python3 bench.py $B > $O/prof.log 2>&1
