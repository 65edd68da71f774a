#!/bin/bash
# A/B of kernel variants on the GPU box: bash tools/gpu_ab.sh spec1 spec2 ...
# (spec = main | <variant>[:KGX_X=v,...]); optional LIST_COUNTERS=1 dumps rocprofv3 -L.
set -o pipefail
mkdir -p gpurun_out
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
if [ -n "$LIST_COUNTERS" ]; then
  (cd /tmp && timeout -k 10 120 rocprofv3 -L) > gpurun_out/counters.txt 2>&1 || echo "counter list failed"
fi
timeout -k 10 900 python tools/exp_agg.py ab "$@" 2>&1 | tee gpurun_out/ab.log
