# Round 6: uneven slice chunks of the push-pull halo (KGX_HALO_WEIGHTS, measurement), NS weak
# P = 8 at a modelled 400 GB/s, share den 32: small first / last chunks against even K 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6w
mkdir -p $O
S="python -u tools/shard_sim.py --config ns --world 8 --steps 10 --exchange halo --free-exchange --link-gbps 400 --share-den 32"
for R in 1 2; do
  timeout -k 10 300 $S --chunks 2 >> $O/w.jsonl 2>> $O/err.log || exit $?
  for W in 1,2 1,3; do
    KGX_HALO_WEIGHTS=$W timeout -k 10 300 $S --chunks 2 >> $O/w.jsonl 2>> $O/err.log || exit $?
  done
  for W in 1,4,1 1,3,1 1,6,1 1,2,1 2,4,1; do
    KGX_HALO_WEIGHTS=$W timeout -k 10 300 $S --chunks 3 >> $O/w.jsonl 2>> $O/err.log || exit $?
  done
  KGX_HALO_WEIGHTS=1,3,3,1 timeout -k 10 300 $S --chunks 4 >> $O/w.jsonl 2>> $O/err.log || exit $?
done
