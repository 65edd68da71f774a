#!/bin/bash
# Round 4: full GPU suite from the current sources, then kgx_dense shapes (the
# producer-epilogue fix) and a short NS bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_gpu_r4.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_r4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_dense.py --reps 20 > gpurun_out/dense_r4.jsonl 2> gpurun_out/dense_r4.err || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ns_r4.json 2> gpurun_out/bench_ns_r4.err
