# Round 6: the owners' pushed partial sums on the fused kernels with W = I (KGX_PARTIAL_FUSED=1)
# against kgx_spmm, one simulated NS weak P = 8 rank at a modelled 400 GB/s (den 32, timelines),
# twice each, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6sim4
mkdir -p $O
S="python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 2 --exchange halo --free-exchange --timeline --link-gbps 400 --share-den 32"
for R in 1 2; do
  timeout -k 10 400 $S > $O/base.$R.jsonl 2>> $O/sim.err || exit $?
  KGX_PARTIAL_FUSED=1 timeout -k 10 400 $S > $O/pfused.$R.jsonl 2>> $O/sim.err || exit $?
done
