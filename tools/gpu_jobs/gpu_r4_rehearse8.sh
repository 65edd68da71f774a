#!/bin/bash
# Round 4: bench.py's N>1 path rehearsed with EIGHT ranks (the driver's node
# size) on one GPU (ranks share cuda:0, exchange staged through host memory over
# gloo, KGX_BENCH_REHEARSAL=1).  At C2's size (1M nodes / 10M edges per rank)
# the first forward stalled past gpurun's 180 s silence limit even with the
# exchange fixed (eight processes multiplexed on one device; 4 ranks had taken
# 126 s), so this runs the "tiny" size (100k / 1M per rank): exchange fixed
# (halo, K 2, unit step), then the tuner (30 s budget).  Progress lines (KGX_LOG)
# on stderr.  Control flow only, never a measurement.
set -o pipefail
mkdir -p gpurun_out/r4r8
O=gpurun_out/r4r8
export TMPDIR=/tmp
KGX_BENCH_REHEARSAL=1 KGX_EXCHANGE=halo KGX_HALO_MERGE=step KGX_HALO_CHUNKS=2 timeout -k 10 400 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus 8 --steps 3 --warmup 1 --config tiny \
  > $O/rehearsal_tiny_n8_fixed.json 2> $O/rehearsal_tiny_n8_fixed.err || exit $?
KGX_BENCH_REHEARSAL=1 KGX_TUNE_BUDGET_S=30 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29539 bench.py --gpus 8 --steps 3 --warmup 1 --config tiny \
  > $O/rehearsal_tiny_n8.json 2> $O/rehearsal_tiny_n8.err || exit $?
