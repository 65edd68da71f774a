# Round 6, first GPU session: the new GCN-norm parity tests (dinv table), the CU-split
# guard, the NS bench line on the changed sources, and one simulated NS weak P = 8 rank
# with the step's timeline (tools/shard_sim.py --timeline) plus the strong-scaled NS rows.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_gcn_norm.py tests/test_gpu_kernels.py tests/test_cu_split_host.py \
  "tests/test_gpu_layers.py::test_hip_graph_capture_cu_split" \
  "tests/test_gpu_distributed.py::test_sharded_aggregation_backward_hip" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_ns.json 2> $O/bench_ns.err || exit $?
timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/bench_ns_train.json 2> $O/bench_ns_train.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o train -- python -u bench.py --train --steps 10 --warmup 2 \
  > $O/prof_train.json 2> $O/prof_train.err || exit $?
