# Round 6: the link probe bench.py uses at N > 1 (asynchronous exchange handles, events on the
# side and probe streams, link_report), exercised through the one-rank simulator's modelled
# link: NS weak P = 8 at 400 GB/s, halo K 2, with and without the probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6probe
mkdir -p $O
timeout -k 10 600 python -u tools/shard_sim.py --config ns --world 8 --chunks 2 --share-den 32 --link-gbps 400 \
  --free-exchange --exchange halo --link-probe --steps 10 > $O/ns_p8_400_probe.jsonl 2> $O/probe.err || exit $?
timeout -k 10 600 python -u tools/shard_sim.py --config ns --world 8 --chunks 2 --share-den 32 --link-gbps 400 \
  --exchange halo --free-exchange --steps 10 > $O/ns_p8_400_noprobe.jsonl 2> $O/noprobe.err || exit $?
