#!/bin/bash
# Round 4 NS weak P=8 one-rank simulations: pass A after the packs
# (KGX_HALO_A_LATE=2) against the layer's rule, compute alone and at modelled
# 400 GB/s (transfer = receive, no local copy).
set -o pipefail
mkdir -p gpurun_out/r4s4
export TMPDIR=/tmp
O=gpurun_out/r4s4
timeout -k 10 600 python tools/shard_sim.py --config ns --world 8 --chunks 1 --merge-unit chunk,step --a-late auto,2 \
  --steps 5 --free-exchange > $O/ns_free.jsonl 2>> $O/sim.err || exit $?
timeout -k 10 600 python tools/shard_sim.py --config ns --world 8 --chunks 1,2 --merge-unit step,chunk --a-late auto,2 \
  --steps 5 --link-gbps 400 --free-exchange > $O/ns_400.jsonl 2>> $O/sim.err || exit $?
