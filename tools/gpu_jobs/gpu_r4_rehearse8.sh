#!/bin/bash
# Round 4: bench.py's N>1 path rehearsed with EIGHT ranks (the driver's node
# size) on one GPU (ranks share cuda:0, exchange staged through host memory over
# gloo, KGX_BENCH_REHEARSAL=1): C2 (weak, 1M nodes / 10M edges per rank) with
# the exchange tuner at the first forward (budget 30 s: host-staged exchanges take
# seconds each).  Control flow only, never a measurement.
set -o pipefail
mkdir -p gpurun_out/r4r8
O=gpurun_out/r4r8
export TMPDIR=/tmp
KGX_BENCH_REHEARSAL=1 KGX_TUNE_BUDGET_S=30 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus 8 --steps 3 --warmup 1 --config c2 \
  > $O/rehearsal_c2_n8.json 2> $O/rehearsal_c2_n8.err || exit $?
