# Round 6: dW / db beside the dx pass (KGX_TN_OVERLAP), the numpy edge_index cache, then the
# sharded NS timeline simulations (tools/gpu_jobs/r6_sim.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_backward.py "tests/test_gpu_layers.py::test_numpy_edge_index_cached" tests/test_gpu_gemm_tn.py \
  > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/bench_ns_train_overlap.json 2> $O/train.err || exit $?
KGX_TN_OVERLAP=0 timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/bench_ns_train_serial.json 2>> $O/train.err || exit $?
bash tools/gpu_jobs/r6_sim.sh
