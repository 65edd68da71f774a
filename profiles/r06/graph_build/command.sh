# Round 6: the graph build's reductions per block instead of per wave (csr_deg, schedule
# suffixes, tiny records): graph-build / tiny / norm tests, then the NS line under a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6build2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_tiny.py tests/test_gpu_gcn_norm.py tests/test_gpu_kernels.py tests/test_gpu_fullsize.py \
  tests/test_gpu_layers.py tests/test_gpu_graph_io.py > $O/pytest.log 2>&1 || exit $?
for R in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_ns.$R.json 2>> $O/bench_ns.err || exit $?
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_ns -o ns \
  -- python -u $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_ns.json 2> $GRAFT_REPO_ROOT/$O/prof_ns.err || exit $?
