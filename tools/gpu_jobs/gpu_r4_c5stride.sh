#!/bin/bash
# Round 4: C5's 400-byte rows -- does the row stride decide the bytes fetched?
# kgx_spmm_ex2 MEAN over the C5 graph with the table at ld 100 / 112 / 128
# (tools/exp_c5_stride.py): time, and FETCH_SIZE per launch (own rocprofv3 pass).
set -o pipefail
mkdir -p gpurun_out/r4st
export TMPDIR=/tmp
O=gpurun_out/r4st
for LD in 100 112 128; do
  timeout -k 10 300 python tools/exp_c5_stride.py --ld $LD >> $O/c5_stride.jsonl 2>> $O/c5.err || exit $?
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$LD -o run \
    --kernel-include-regex spmm -- python3 tools/exp_c5_stride.py --ld $LD --reps 3 > $O/pmc_$LD.log 2>&1 || exit $?
done
