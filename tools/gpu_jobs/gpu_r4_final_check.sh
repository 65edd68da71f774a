#!/bin/bash
# Round 4, last check from the final tree: the GPU suite, smoke(), the driver's
# own bench command (N=1), and bench.py's N>1 path at N=2 (tiny size, one GPU,
# host-staged gloo; control flow of the final bench.py / distributed.py).
set -o pipefail
mkdir -p gpurun_out/r4fc
export TMPDIR=/tmp
O=gpurun_out/r4fc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit $?
KGX_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 3 --warmup 1 --config tiny \
  > $O/rehearsal_tiny_n2.json 2> $O/rehearsal_tiny_n2.err || exit $?
