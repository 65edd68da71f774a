#!/bin/bash
# Round 4: EXACT mode with the hub kernel forked beside spmm_kernel, which keeps
# its full grid and takes interleaved row batches from a counter
# (KGX_EXACT_FORK=3), against the sequential default; NS --exact interleaved,
# after the EXACT / bit-identity GPU tests under the fork.
set -o pipefail
mkdir -p gpurun_out/r4f3
export TMPDIR=/tmp
O=gpurun_out/r4f3
KGX_EXACT_FORK=3 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
  -k "exact or bitwise or bit_identical" --timeout 240 --timeout-method thread > $O/pytest_fork3.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_fork3.log
[ $rc -eq 0 ] || exit $rc
B="--exact --steps 20 --warmup 3 --no-cpu-baseline --no-cold"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/exact_f0_r$r.json 2>> $O/bench.err || exit $?
  KGX_EXACT_FORK=3 timeout -k 10 300 python bench.py $B > $O/exact_f3_r$r.json 2>> $O/bench.err || exit $?
done
KGX_EXACT_FORK=3 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python3 bench.py $B > $O/prof.log 2>&1
