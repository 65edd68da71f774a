# Round 3: full GPU suite, then the north-star bench + rocprofv3 stats + PMC traffic.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
bash profiles/r03/command_ns.sh || exit $?
cat gpurun_out/bench_ns.json
