#!/bin/bash
# Round 4: full GPU suite from the current sources, kgx_dense shapes (producer
# epilogue fix), NS bench line, and the C4 strong P=8 one-rank simulation with the
# fused two-table 256-wide passes (ShardedGINConv); C5 with the fused SAGE update.
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
# C5: SAGE update fused into the aggregation (kgx_spmm_gemm at F 100) vs the two-step path
timeout -k 10 400 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-cold \
  > gpurun_out/r4/bench_c5.json 2> gpurun_out/r4/bench_c5.err || exit $?
KGX_FUSED_SAGE=0 timeout -k 10 400 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-cold \
  > gpurun_out/r4/bench_c5_unfused.json 2>> gpurun_out/r4/bench_c5.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4/c5_trace -o run \
  -- python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/r4/c5_trace.log 2>&1
