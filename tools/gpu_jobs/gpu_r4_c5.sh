#!/bin/bash
# Round 4: the GPU suite, then same-box A/B runs (interleaved, two rounds):
# NS GCN layer; C5 SAGEConv mean with the fused update (narrow kernels, main
# kernel U = 6) against KGX_TINY_ACC_EARLY=1 (libkgx_accearly.so) and the
# two-step path (KGX_FUSED_SAGE=0); rocprofv3 kernel stats of the fused C5 layer.
# Build first (here): make -C keras-geometric_amd/csrc variant NAME=accearly DEFS=-DKGX_TINY_ACC_EARLY=1
set -o pipefail
mkdir -p gpurun_out/r4c5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  > gpurun_out/r4c5/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4c5/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
V=keras-geometric_amd/lib/variants
B="--no-cpu-baseline --no-cold"
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 $B > gpurun_out/r4c5/ns_r$r.json 2>> gpurun_out/r4c5/bench.err || exit $?
  timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 $B > gpurun_out/r4c5/fused_r$r.json 2>> gpurun_out/r4c5/bench.err || exit $?
  KGX_LIB=$V/libkgx_accearly.so timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 $B \
    > gpurun_out/r4c5/accearly_r$r.json 2>> gpurun_out/r4c5/bench.err || exit $?
  KGX_FUSED_SAGE=0 timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 $B \
    > gpurun_out/r4c5/twostep_r$r.json 2>> gpurun_out/r4c5/bench.err || exit $?
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4c5/prof -o run \
  -- python3 bench.py --config c5 --steps 10 --warmup 2 $B > gpurun_out/r4c5/prof.log 2>&1 || exit $?
KGX_FUSED_SAGE=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4c5/prof2 -o run \
  -- python3 bench.py --config c5 --steps 10 --warmup 2 $B > gpurun_out/r4c5/prof2.log 2>&1
