#!/bin/bash
# Round 4: C4 GIN layer, the 256-wide kernels loading the rows' own x rows with
# the next tile's prefetch (KGX_F256_ROOT_PF=1) against the shipped form, interleaved;
# the 256-wide tests under the variant first.
# Build first (here): make -C keras-geometric_amd/csrc variant NAME=rootpf DEFS=-DKGX_F256_ROOT_PF=1
set -o pipefail
mkdir -p gpurun_out/r4rp
export TMPDIR=/tmp
O=gpurun_out/r4rp
V=keras-geometric_amd/lib/variants/libkgx_rootpf.so
KGX_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_fused256.py -x -q -p no:cacheprovider --timeout 240 \
  --timeout-method thread > $O/pytest_rootpf.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_rootpf.log
[ $rc -eq 0 ] || exit $rc
B="--config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-cold"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/c4_ship_r$r.json 2>> $O/bench.err || exit $?
  KGX_LIB=$V timeout -k 10 300 python bench.py $B > $O/c4_rootpf_r$r.json 2>> $O/bench.err || exit $?
done
KGX_LIB=$V timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python3 bench.py $B > $O/prof.log 2>&1
