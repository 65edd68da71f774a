# Round 6: dW (kgx_gemm_tn) forked after the dx launch (W^T no longer queued behind it):
# the NS training step with LDS / register dW forms and with the overlap off, then a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ovl2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_gemm_tn.py tests/test_gpu_backward.py > $O/pytest.log 2>&1 || exit $?
for R in 1 2; do
  timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_lds.$R.json 2>> $O/train.err || exit $?
  KGX_TN_LDS=0 timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_reg.$R.json 2>> $O/train.err || exit $?
  KGX_TN_OVERLAP=0 timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_serial.$R.json 2>> $O/train.err || exit $?
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o train \
  -- python -u $GRAFT_REPO_ROOT/bench.py --train --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof_train.json 2> $GRAFT_REPO_ROOT/$O/prof.err || exit $?
