# Round 6: the graph build with the source carried through the sort and the tail records built
# on the device: parity tests, then the NS bench line under a kernel trace (build breakdown).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_tiny.py tests/test_gpu_gcn_norm.py tests/test_gpu_kernels.py tests/test_gpu_fullsize.py \
  tests/test_gpu_layers.py tests/test_gpu_graph_io.py > $O/pytest.log 2>&1 || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_ns -o ns \
  -- python -u $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/bench_ns.json 2> $GRAFT_REPO_ROOT/$O/bench_ns.err || exit $?
