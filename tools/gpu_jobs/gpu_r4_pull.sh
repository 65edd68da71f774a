#!/bin/bash
# Round 4: the pull-only halo through the merged passes (exchange kind "pull":
# every halo edge served by pulling its source, no partial sums) against the
# push-pull halo ("halo") in the NS weak P=8 one-rank simulation, compute alone
# (--free-exchange) and at modelled 400 GB/s (transfer = receive).  Push-pull
# moves 45 % fewer rows but the owner computes and writes the pushed partial
# sums (2.1 + 0.9 ms of short-row passes in the round-4 trace); the tuner now
# times both.
set -o pipefail
mkdir -p gpurun_out/r4pl
export TMPDIR=/tmp
O=gpurun_out/r4pl
for r in 1 2; do
  timeout -k 10 600 python tools/shard_sim.py --config ns --world 8 --exchange halo,pull --chunks 1,2 \
    --merge-unit chunk,step --steps 5 --free-exchange >> $O/ns_free.jsonl 2>> $O/sim.err || exit $?
done
timeout -k 10 600 python tools/shard_sim.py --config ns --world 8 --exchange halo,pull --chunks 1,2 \
  --merge-unit chunk,step --steps 5 --link-gbps 400 --free-exchange >> $O/ns_400.jsonl 2>> $O/sim.err || exit $?
