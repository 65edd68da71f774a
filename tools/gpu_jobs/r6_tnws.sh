# Round 6: kgx_gemm_tn warp-specialised form (KGX_TN_LDS=2, default) against the LDS form (1):
# gemm_tn tests under each, standalone timing, the NS training step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6tnws
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_gemm_tn.py tests/test_gpu_backward.py > $O/pytest_ws.log 2>&1 || exit $?
for R in 1 2; do
  timeout -k 10 120 python -u tools/exp_gemm_tn.py >> $O/tn.jsonl 2>> $O/err.log || exit $?
  KGX_TN_LDS=1 timeout -k 10 120 python -u tools/exp_gemm_tn.py >> $O/tn.jsonl 2>> $O/err.log || exit $?
done
for R in 1 2; do
  timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_ws.$R.json 2>> $O/train.err || exit $?
  KGX_TN_LDS=1 timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_lds.$R.json 2>> $O/train.err || exit $?
done
