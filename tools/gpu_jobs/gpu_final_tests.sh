# Round-end check: the whole GPU test suite, then smoke().
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/full.log 2>&1 || { tail -30 gpurun_out/full.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/full.log; cat gpurun_out/smoke.log | tail -2
