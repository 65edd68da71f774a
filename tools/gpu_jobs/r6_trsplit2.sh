# Round 6: the training backward's transposed pass one-stream (ops._unsplit, default) against
# the CU split kept (KGX_BWD_CU_SPLIT=1); backward tests; a kernel trace of the default step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6trsplit2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_backward.py tests/test_gpu_gemm_tn.py > $O/pytest.log 2>&1 || exit $?
for R in 1 2 3; do
  timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_default.$R.json 2>> $O/err.log || exit $?
  KGX_BWD_CU_SPLIT=1 timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_bwdsplit.$R.json 2>> $O/err.log || exit $?
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace_train -o run \
  -- python3 $GRAFT_REPO_ROOT/bench.py --train --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/$O/trace_train.log 2>&1 || exit $?
