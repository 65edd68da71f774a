# Round 6: the one-pass dW / db kernel (kgx_gemm_tn): its tests, the backward suite,
# and the NS training step (bench.py --train) with a rocprofv3 kernel-stats summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_gemm_tn.py tests/test_gpu_backward.py tests/test_gpu_dense.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/bench_ns_train.json 2> $O/bench_ns_train.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_train -o train \
  -- python -u $GRAFT_REPO_ROOT/bench.py --train --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof_train.json 2> $GRAFT_REPO_ROOT/$O/prof_train.err || exit $?
