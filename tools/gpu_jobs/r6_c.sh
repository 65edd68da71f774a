# Round 6: the fused col + norm graph-build pass and the long-row edge-norm kernel: the CSR /
# GCN-norm parity tests, the sharded GCN tests that use the edge-norm kernel, and the NS bench
# line under a rocprofv3 kernel trace (graph build breakdown: tools/build_breakdown.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_gcn_norm.py tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py \
  "tests/test_gpu_layers.py::test_numpy_edge_index_cached" > $O/pytest.log 2>&1 || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_ns -o ns \
  -- python -u $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/bench_ns.json 2> $GRAFT_REPO_ROOT/$O/bench_ns.err || exit $?
