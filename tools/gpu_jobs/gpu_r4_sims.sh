#!/bin/bash
# Round 4 one-rank simulations (tools/shard_sim.py): C4 GIN-sum strong P=8 with
# the fused two-table 256-wide passes (exchange-free: loopback copy and free;
# modelled 400 GB/s links), and NS GCN weak P=8 at modelled 400 GB/s links.
set -o pipefail
mkdir -p gpurun_out/r4s
export TMPDIR=/tmp
O=gpurun_out/r4s
timeout -k 10 400 python tools/shard_sim.py --config c4 --world 8 --exchange halo --chunks 1,2 --steps 5 \
  > $O/c4_p8.jsonl 2>> $O/sim.err || exit $?
timeout -k 10 400 python tools/shard_sim.py --config c4 --world 8 --exchange halo --chunks 1 --steps 5 --free-exchange \
  >> $O/c4_p8.jsonl 2>> $O/sim.err || exit $?
timeout -k 10 400 python tools/shard_sim.py --config c4 --world 8 --exchange halo --chunks 1,2 --steps 5 --link-gbps 400 \
  >> $O/c4_p8.jsonl 2>> $O/sim.err || exit $?
timeout -k 10 600 python tools/shard_sim.py --config ns --world 8 --chunks 1,2 --merge-unit chunk,step --steps 5 \
  --link-gbps 400 > $O/ns_p8_400.jsonl 2>> $O/sim.err || exit $?
