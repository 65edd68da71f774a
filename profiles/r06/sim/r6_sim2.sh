# Round 6: the dual-stream merged passes (KGX_HALO_DUAL=1) against the one-stream default, one
# simulated NS weak P = 8 rank at a modelled 400 GB/s with timelines, share den 16 / 32; and the
# threaded-rank GPU tests of the dual path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6sim2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py -k "dual or chunked_halo" > $O/pytest.log 2>&1 || exit $?
S="python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 2 --exchange halo --free-exchange --timeline --link-gbps 400"
KGX_HALO_DUAL=1 timeout -k 10 600 $S --share-den 16,32 > $O/ns_p8_400_dual.jsonl 2> $O/sim.err || exit $?
timeout -k 10 600 $S --share-den 16,32 > $O/ns_p8_400_base.jsonl 2>> $O/sim.err || exit $?
KGX_HALO_DUAL=1 KGX_HALO_FIRST=0.3 timeout -k 10 600 $S --share-den 16 > $O/ns_p8_400_dual_first03.jsonl 2>> $O/sim.err || exit $?
