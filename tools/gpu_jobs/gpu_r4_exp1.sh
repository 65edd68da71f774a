#!/bin/bash
# Round 4 experiments: (1) EXACT mode, hub kernel forked beside a static
# interleaved spmm_kernel (KGX_EXACT_FORK=2) vs the sequential default, A/B
# interleaved, plus the bit-identity test under the fork; (2) NS weak P=8
# one-rank simulation: KGX_SHARE_DEN sweep (loopback-copy exchange), the compute-only step
# (--free-exchange) per merge unit and pass order, and a rocprofv3 kernel trace (pack / pass A / pass B).
set -o pipefail
mkdir -p gpurun_out/r4x
export TMPDIR=/tmp
for r in 1 2; do
  for M in "0 0" "2 0" "2 128"; do
    set -- $M
    KGX_EXACT_FORK=$1 KGX_EXACT_HUB_CUS=$2 timeout -k 10 300 python bench.py --exact --steps 20 --warmup 3 \
      --no-cpu-baseline --no-cold > gpurun_out/r4x/exact_f$1_c$2_r$r.json 2>> gpurun_out/r4x/exact.err || exit $?
  done
done
KGX_EXACT_FORK=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -q -x -p no:cacheprovider \
  -k "exact_aggregation_bitwise" --timeout 240 --timeout-method thread > gpurun_out/r4x/exact_fork_test.log 2>&1 || exit $?
timeout -k 10 900 python tools/shard_sim.py --config ns --world 8 --chunks 1 --merge-unit chunk --steps 5 \
  --share-den 8,4,2,16 > gpurun_out/r4x/sim_ns_share.jsonl 2> gpurun_out/r4x/sim_ns_share.err || exit $?
timeout -k 10 900 python tools/shard_sim.py --config ns --world 8 --chunks 1 --merge-unit chunk,step --a-late 0,1 \
  --steps 5 --share-den 8,4 --free-exchange > gpurun_out/r4x/sim_ns_free.jsonl 2> gpurun_out/r4x/sim_ns_free.err || exit $?
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4x/sim_ns -o run \
  -- python3 tools/shard_sim.py --config ns --world 8 --chunks 1 --merge-unit chunk --steps 5 \
  > gpurun_out/r4x/sim_ns.jsonl 2> gpurun_out/r4x/sim_ns.err
