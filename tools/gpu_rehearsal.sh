#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box: N ranks share cuda:0 and the
# halo exchange is staged through host memory over gloo (KGX_BENCH_REHEARSAL=1).
# Checks the multi-rank control flow end to end; the timings mean nothing.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for n in 2 4; do
  KGX_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29510 + n)) bench.py --gpus $n --steps 3 --warmup 1 --config c2 \
    > gpurun_out/rehearsal$n.json 2> gpurun_out/rehearsal$n.err || exit $?
done
