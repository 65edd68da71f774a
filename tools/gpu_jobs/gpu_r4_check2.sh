#!/bin/bash
# Round 4 (second half of the check): the C4 strong P=8 one-rank simulation with the fused
# two-table 256-wide passes (ShardedGINConv), and C5's row stride vs bytes fetched.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
for L in 0 400; do
  timeout -k 10 400 python tools/shard_sim.py --config c4 --world 8 --exchange halo --chunks 1,2 \
    --link-gbps $L --steps 5 >> gpurun_out/r4/c4_p8.jsonl 2>> gpurun_out/r4/sim.err || exit $?
done
# C5: row stride vs bytes fetched (400 / 448 / 512-byte rows), and the layer's kernel timeline
for LD in 100 112 128; do
  timeout -k 10 300 python tools/exp_c5_stride.py --ld $LD >> gpurun_out/r4/c5_stride.jsonl 2>> gpurun_out/r4/c5.err || exit $?
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4/c5_pmc_$LD -o run \
    --kernel-include-regex spmm -- python3 tools/exp_c5_stride.py --ld $LD --reps 3 > gpurun_out/r4/c5_pmc_$LD.log 2>&1 || exit $?
done
