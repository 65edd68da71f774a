#!/bin/bash
# Round 4: the 256-wide fused kernels with the f16x2 split (KGX_F256_SPLIT=2, the
# new default in libkgx.so) against bf16x3 (variant b3), C4 GIN layer interleaved;
# the 256-wide / C4 / GIN tests under the new default first, kernel stats after.
# Build first (here): make -C keras-geometric_amd/csrc variant NAME=b3 DEFS=-DKGX_F256_SPLIT=3
set -o pipefail
mkdir -p gpurun_out/r4h2
export TMPDIR=/tmp
O=gpurun_out/r4h2
V=keras-geometric_amd/lib/variants/libkgx_b3.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused256.py -x -v -p no:cacheprovider --timeout 240 \
  --timeout-method thread > $O/pytest_h2.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_h2.log
[ $rc -eq 0 ] || exit $rc
B="--config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-cold"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/c4_h2_r$r.json 2>> $O/bench.err || exit $?
  KGX_LIB=$V timeout -k 10 300 python bench.py $B > $O/c4_b3_r$r.json 2>> $O/bench.err || exit $?
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python3 bench.py $B > $O/prof.log 2>&1
