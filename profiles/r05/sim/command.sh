# Round 5: one rank of NS weak P = 8 (tools/shard_sim.py): the slice-chunked push-pull
# halo (K 2, unit step: round 4's best at modelled 400 GB/s) against the destination-
# group chunks (exchange "group", K 2 / 3 / 4, with and without a small first group),
# compute alone and at a modelled 400 GB/s (transfer time = the receive).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5sim
mkdir -p $O
S="python -u tools/shard_sim.py --config ns --world 8 --steps 10"
timeout -k 10 400 $S --chunks 2 --exchange halo --free-exchange > $O/free_halo.jsonl 2> $O/err.log || exit $?
timeout -k 10 400 $S --chunks 2,4 --exchange group --free-exchange > $O/free_group.jsonl 2>> $O/err.log || exit $?
timeout -k 10 400 $S --chunks 2 --exchange halo --free-exchange --link-gbps 400 > $O/l400_halo.jsonl 2>> $O/err.log || exit $?
timeout -k 10 500 $S --chunks 2,3,4 --exchange group --free-exchange --link-gbps 400 > $O/l400_group.jsonl 2>> $O/err.log || exit $?
KGX_HALO_FIRST=0.15 timeout -k 10 400 $S --chunks 3,4 --exchange group --free-exchange --link-gbps 400 > $O/l400_group_first.jsonl 2>> $O/err.log || exit $?
# C4 GIN-sum strong P = 8 (fused 256-wide passes): slice chunks vs destination groups at 400 GB/s
C="python -u tools/shard_sim.py --config c4 --world 8 --steps 10"
timeout -k 10 400 $C --chunks 1,2 --exchange halo --merge-unit chunk,step --free-exchange --link-gbps 400 > $O/c4_l400_halo.jsonl 2>> $O/err.log || exit $?
timeout -k 10 400 $C --chunks 2,3,4 --exchange group --free-exchange --link-gbps 400 > $O/c4_l400_group.jsonl 2>> $O/err.log || exit $?
timeout -k 10 400 $C --chunks 2,4 --exchange group --free-exchange > $O/c4_free_group.jsonl 2>> $O/err.log || exit $?
