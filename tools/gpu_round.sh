#!/bin/bash
# Full GPU pass: pytest -m gpu, then the north-star bench + rocprofv3 passes.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_check.sh || exit $?
grep -q "pytest rc=0" gpurun_out/pytest_gpu.log || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
bash tools/gpu_bench.sh
