# Round 5: the pruned push-pull plan (default) confirmed on a second box: NS weak P = 8, halo K 2,
# modelled 400 GB/s, share den 16 (default) and 32, two rounds -> gpurun_out/prune2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/prune2
mkdir -p $O
for round in 1 2; do
  timeout -k 10 400 python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 2 --exchange halo --free-exchange --link-gbps 400 --share-den 16,32 > $O/ns_prune_den.$round.jsonl 2>> $O/err.log || exit $?
done
