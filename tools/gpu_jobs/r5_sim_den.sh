# Round 5: with light rows, the block-slot share the passes leave the exchange (KGX_SHARE_DEN 4 / 8 / 16),
# NS weak P = 8, halo K 2 step, 400 GB/s, two rounds -> gpurun_out/r5sd2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5sd2
mkdir -p $O
for round in 1 2; do
  timeout -k 10 400 python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 2 --exchange halo --free-exchange --link-gbps 400 --share-den 16,32,64,1000 > $O/den.$round.jsonl 2>> $O/err.log || exit $?
done
