#!/bin/bash
# Round 4 one-rank simulations at modelled 400 GB/s links with the transfer time
# standing for RCCL's receive (--free-exchange: no local copy after the first
# landing): NS GCN weak P=8 and C4 GIN-sum strong P=8 over K x merge unit x order.
set -o pipefail
mkdir -p gpurun_out/r4s3
export TMPDIR=/tmp
O=gpurun_out/r4s3
timeout -k 10 600 python tools/shard_sim.py --config ns --world 8 --chunks 1,2,4 --merge-unit step,chunk --a-late 0,1 \
  --steps 5 --link-gbps 400 --free-exchange > $O/ns_p8_400_free.jsonl 2>> $O/sim.err || exit $?
timeout -k 10 400 python tools/shard_sim.py --config c4 --world 8 --chunks 1,2 --merge-unit step,chunk \
  --steps 5 --link-gbps 400 --free-exchange > $O/c4_p8_400_free.jsonl 2>> $O/sim.err || exit $?
