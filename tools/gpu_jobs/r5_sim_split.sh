# Round 5: NS weak P = 8 and C4 strong P = 8 shard simulations (halo K 2, unit step, 400 GB/s
# modelled link) with the CU split off / default rule / forced on every pass incl. the ones
# sharing the GPU with the exchange -> gpurun_out/r5ss
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5ss
mkdir -p $O
S="python -u tools/shard_sim.py --world 8 --steps 10 --chunks 2 --exchange halo --free-exchange --link-gbps 400"
for round in 1 2; do
  KGX_FUSED_CU_SPLIT=0 KGX_F256_CU_SPLIT=0 timeout -k 10 300 $S --config ns > $O/ns_off.$round.jsonl 2>> $O/err.log || exit $?
  timeout -k 10 300 $S --config ns > $O/ns_default.$round.jsonl 2>> $O/err.log || exit $?
  KGX_FUSED_CU_SPLIT=8 KGX_CU_SPLIT_SHARED=1 timeout -k 10 300 $S --config ns > $O/ns_forced.$round.jsonl 2>> $O/err.log || exit $?
done
KGX_F256_CU_SPLIT=0 timeout -k 10 300 $S --config c4 > $O/c4_off.jsonl 2>> $O/err.log || exit $?
KGX_F256_CU_SPLIT=8 KGX_CU_SPLIT_SHARED=1 timeout -k 10 300 $S --config c4 > $O/c4_forced.jsonl 2>> $O/err.log || exit $?
