# Round 6: one simulated NS weak P = 8 rank (tools/shard_sim.py) with the step's timeline,
# at a modelled 400 GB/s (share den 16 / 32) and compute alone, plus the strong-scaled
# NS rows (the one 10M / 100M graph over P = 2 / 4 / 8).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6sim
mkdir -p $O
S="python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 2 --exchange halo --free-exchange --timeline"
timeout -k 10 500 $S --link-gbps 400 --share-den 16,32 > $O/sim_ns_p8_400.jsonl 2> $O/sim.err || exit $?
timeout -k 10 500 $S --share-den 16 > $O/sim_ns_p8_free.jsonl 2>> $O/sim.err || exit $?
T="python -u tools/shard_sim.py --config ns_strong --steps 10 --exchange halo --free-exchange --link-gbps 400"
for P in 2 4 8; do
  timeout -k 10 400 $T --world $P --chunks 1,2 --share-den 16 > $O/sim_nsstrong_p$P.jsonl 2>> $O/sim.err || exit $?
done
