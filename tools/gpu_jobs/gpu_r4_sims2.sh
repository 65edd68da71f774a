#!/bin/bash
# Round 4 one-rank simulations, second sweep: C4 GIN-sum strong P=8 compute-only
# step (--free-exchange) over merge unit x KGX_SHARE_DEN x pass order, with a
# kernel trace; NS GCN weak P=8 at modelled 400 GB/s over K x merge unit x share.
set -o pipefail
mkdir -p gpurun_out/r4s2
export TMPDIR=/tmp
O=gpurun_out/r4s2
timeout -k 10 400 python tools/shard_sim.py --config c4 --world 8 --chunks 1,2 --merge-unit step,chunk --a-late 0,1 \
  --share-den 8,4,2 --steps 5 --free-exchange > $O/c4_p8_free.jsonl 2>> $O/sim.err || exit $?
timeout -k 10 600 python tools/shard_sim.py --config ns --world 8 --chunks 2,4 --merge-unit step,chunk --a-late 0,1 \
  --share-den 8,4 --steps 5 --link-gbps 400 > $O/ns_p8_400.jsonl 2>> $O/sim.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/c4_trace -o run \
  -- python3 tools/shard_sim.py --config c4 --world 8 --chunks 1 --steps 5 --free-exchange > $O/c4_trace.log 2>&1
