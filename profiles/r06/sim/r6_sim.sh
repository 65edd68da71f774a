# Round 6: one simulated NS weak P = 8 rank (tools/shard_sim.py) with the step's timeline at a
# modelled 400 GB/s: the round-5 default (pass A after the merged pass) against pass A first
# after the first step's packing (KGX_HALO_A_LATE=3), share den 16 / 32, and a small first
# chunk; then the strong-scaled NS rows (the one 10M / 100M graph over P = 2 / 4 / 8).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6sim
mkdir -p $O
S="python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 2 --exchange halo --free-exchange --timeline --link-gbps 400"
timeout -k 10 600 $S --share-den 16,32 --a-late auto,3 > $O/ns_p8_400_alate.jsonl 2> $O/sim.err || exit $?
KGX_HALO_FIRST=0.3 timeout -k 10 400 $S --share-den 16 --a-late auto,3 > $O/ns_p8_400_first03.jsonl 2>> $O/sim.err || exit $?
