# Round 6: one simulated NS weak P = 8 rank at a modelled 400 GB/s: halo K 2 / 3 x merge unit
# step / chunk at share den 32 (light rows and pruned pulls on); then the strong-scaled NS rows
# (the one 10M / 100M graph over P = 2 / 4 / 8 ranks, halo K 1 / 2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6sim3
mkdir -p $O
S="python -u tools/shard_sim.py --config ns --world 8 --steps 10 --exchange halo --free-exchange --link-gbps 400"
timeout -k 10 800 $S --chunks 2,3 --merge-unit step,chunk --share-den 32 > $O/ns_p8_400_units.jsonl 2> $O/sim.err || exit $?
timeout -k 10 400 $S --chunks 2 --share-den 16,32 --link-gbps 0 > $O/ns_p8_free.jsonl 2>> $O/sim.err || exit $?
T="python -u tools/shard_sim.py --config ns_strong --steps 10 --exchange halo --free-exchange --link-gbps 400"
for P in 2 4 8; do
  timeout -k 10 400 $T --world $P --chunks 1,2 --share-den 16,32 > $O/nsstrong_p$P.jsonl 2>> $O/sim.err || exit $?
done
