# Round 6: kgx_gemm_tn's LDS form (split once per block, transposed LDS reads) against the
# per-wave split form (KGX_TN_LDS=0): tests, then the NS training step with each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6tn
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_gemm_tn.py tests/test_gpu_backward.py > $O/pytest.log 2>&1 || exit $?
KGX_TN_LDS=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_gemm_tn.py > $O/pytest_tn0.log 2>&1 || exit $?
for R in 1 2; do
  timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_lds.$R.json 2>> $O/train.err || exit $?
  KGX_TN_LDS=0 timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_reg.$R.json 2>> $O/train.err || exit $?
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o train \
  -- python -u $GRAFT_REPO_ROOT/bench.py --train --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof_train.json 2> $GRAFT_REPO_ROOT/$O/prof.err || exit $?
