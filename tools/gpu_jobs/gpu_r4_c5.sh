#!/bin/bash
# Round 4, C5 (SAGEConv mean, 2.45M / 123.7M, F 100) with the fused update:
# (1) interleaved A/B of the shipped library against KGX_TINY_ACC_EARLY=1
# (lib/variants/libkgx_accearly.so: the tiny kernel's accumulate loads issued
# before its MFMAs) and against the two-step path (KGX_FUSED_SAGE=0);
# (2) rocprofv3 kernel stats + trace of the fused C5 layer (per-kernel times,
# idle time between launches: tools/trace_gaps.py).
set -o pipefail
mkdir -p gpurun_out/r4c5
export TMPDIR=/tmp
V=keras-geometric_amd/lib/variants/libkgx_accearly.so
for r in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-cold \
    > gpurun_out/r4c5/fused_r$r.json 2>> gpurun_out/r4c5/bench.err || exit $?
  KGX_LIB=$V timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-cold \
    > gpurun_out/r4c5/accearly_r$r.json 2>> gpurun_out/r4c5/bench.err || exit $?
  KGX_FUSED_SAGE=0 timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-cold \
    > gpurun_out/r4c5/twostep_r$r.json 2>> gpurun_out/r4c5/bench.err || exit $?
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4c5/prof -o run \
  -- python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/r4c5/prof.log 2>&1
