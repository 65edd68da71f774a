# Round 5: push-pull plan with and without dropping pulled sources whose rows are all pushed anyway
# (KGX_HALO_PRUNE=1 / 0), one simulated rank at a modelled 400 GB/s: NS weak P = 8 (halo K 2) and
# C4 strong P = 8 (halo K 1), two rounds, interleaved -> gpurun_out/prune
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/prune
mkdir -p $O
for round in 1 2; do
  for p in 0 1; do
    KGX_HALO_PRUNE=$p timeout -k 10 400 python -u tools/shard_sim.py --config c4 --world 8 --steps 10 --chunks 1 --exchange halo --free-exchange --link-gbps 400 --share-den 16 > $O/c4_prune$p.$round.jsonl 2>> $O/err.log || exit $?
    KGX_HALO_PRUNE=$p timeout -k 10 400 python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 2 --exchange halo --free-exchange --link-gbps 400 --share-den 16 > $O/ns_prune$p.$round.jsonl 2>> $O/err.log || exit $?
  done
done
