# Round 5: bench.py's N > 1 path rehearsed on one GPU (ranks share cuda:0, exchange
# staged through host memory over gloo): N = 2 at C2's size (tuner incl. the
# destination-group candidates) and N = 2 with the C4 GIN layer -> gpurun_out/reh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/reh
mkdir -p $O
KGX_BENCH_REHEARSAL=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --config c2 \
  > $O/rehearsal_c2_n2.json 2> $O/rehearsal_c2_n2.err || exit $?
KGX_BENCH_REHEARSAL=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --steps 3 --warmup 1 --config tiny \
  > $O/rehearsal_tiny_n2.json 2> $O/rehearsal_tiny_n2.err || exit $?
