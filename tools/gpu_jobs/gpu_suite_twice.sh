# The whole GPU suite twice in one call (flakiness check), then smoke().
set -o pipefail
mkdir -p gpurun_out
for n in 1 2; do
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/full_$n.log 2>&1
  echo "run $n rc=$?"; tail -1 gpurun_out/full_$n.log; grep FAILED gpurun_out/full_$n.log | head -5
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
