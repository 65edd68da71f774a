# Round 6: bench.py's N = 2 path rehearsed on one GPU (ranks share cuda:0, host-staged gloo
# exchange): the self-checking line (per-rank roofline, links, halo bytes), GCN C2 and NS weak.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6reh2
mkdir -p $O
KGX_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --config c2 \
  > $O/rehearsal_c2_n2.json 2> $O/rehearsal_c2_n2.err || exit $?
