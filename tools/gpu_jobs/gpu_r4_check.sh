#!/bin/bash
# Round 4: full GPU suite from the current sources, kgx_dense shapes (producer
# epilogue fix), NS bench line, and the C4 strong P=8 one-rank simulation with the
# fused two-table 256-wide passes (ShardedGINConv).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  > gpurun_out/r4/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_dense.py --reps 20 > gpurun_out/r4/dense.jsonl 2> gpurun_out/r4/dense.err || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r4/bench_ns.json 2> gpurun_out/r4/bench_ns.err || exit $?
for L in 0 400; do
  timeout -k 10 400 python tools/shard_sim.py --config c4 --world 8 --exchange halo --chunks 1,2 \
    --link-gbps $L --steps 5 >> gpurun_out/r4/c4_p8.jsonl 2>> gpurun_out/r4/sim.err || exit $?
done
