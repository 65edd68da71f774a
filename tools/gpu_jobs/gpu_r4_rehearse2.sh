#!/bin/bash
# Round 4: bench.py's N>1 path rehearsed on one GPU for the strong-scaled configs
# (ranks share cuda:0, exchange staged through host memory over gloo): C4 GIN-sum
# (fused two-table 256-wide passes) and C5 SAGE-mean at N=2.  Control flow only.
set -o pipefail
mkdir -p gpurun_out/r4r2
O=gpurun_out/r4r2
export TMPDIR=/tmp
for c in c4 c5; do
  KGX_BENCH_REHEARSAL=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --config $c \
    > $O/rehearsal_${c}_n2.json 2> $O/rehearsal_${c}_n2.err || exit $?
done
