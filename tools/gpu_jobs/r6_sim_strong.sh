# Round 6: strong-scaled NS (the one 10M / 100M graph over P = 2 / 4 / 8 ranks), one simulated
# rank each at a modelled 400 GB/s, halo K 1 / 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6sim
mkdir -p $O
T="python -u tools/shard_sim.py --config ns_strong --steps 10 --exchange halo --free-exchange --link-gbps 400"
for P in 2 4 8; do
  timeout -k 10 400 $T --world $P --chunks 1,2 --share-den 16 > $O/nsstrong_p$P.jsonl 2>> $O/sim_strong.err || exit $?
done
