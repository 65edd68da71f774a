#!/bin/bash
# A/B timing of variants + LDS bank-conflict counter per variant.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/abpmc
export TMPDIR=/tmp
timeout -k 10 900 python tools/exp_agg.py ab "$@" 2>&1 | tee gpurun_out/ab.log || exit $?
for spec in "$@"; do
  name=${spec%%:*}
  lib=$PWD/keras-geometric_amd/lib/libkgx.so
  [ "$name" != "main" ] && lib=$PWD/keras-geometric_amd/lib/variants/libkgx_$name.so
  KGX_LIB=$lib timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv \
    -d gpurun_out/abpmc/$name -o run --kernel-include-regex spmm_gemm_kernel -- python3 tools/exp_agg.py both \
    > gpurun_out/abpmc/$name.log 2>&1 || exit $?
done
