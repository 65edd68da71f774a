#!/bin/bash
# Round 4: bench.py's N>1 path rehearsed on one GPU (ranks share cuda:0, exchange
# staged through host memory over gloo, KGX_BENCH_REHEARSAL=1): C2 at N=2 and 4,
# and the north-star config (NS weak scaling) at N=2.  Control flow only.
set -o pipefail
mkdir -p gpurun_out/r4r
O=gpurun_out/r4r
export TMPDIR=/tmp
for n in 2 4; do
  KGX_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29510 + n)) bench.py --gpus $n --steps 3 --warmup 1 --config c2 \
    > $O/rehearsal_c2_n$n.json 2> $O/rehearsal_c2_n$n.err || exit $?
done
KGX_BENCH_REHEARSAL=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29520 bench.py --gpus 2 --steps 3 --warmup 1 \
  > $O/rehearsal_ns_n2.json 2> $O/rehearsal_ns_n2.err || exit $?
