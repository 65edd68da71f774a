# Round 6: kgx_gemm_tn warp-specialised form with five steps of loads in flight (KGX_TN_SETS=6)
# against three (default): gemm_tn tests under 6, standalone timing, the NS training step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6tnsets
mkdir -p $O
KGX_TN_SETS=6 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_gemm_tn.py > $O/pytest6.log 2>&1 || exit $?
for R in 1 2 3; do
  timeout -k 10 120 python -u tools/exp_gemm_tn.py >> $O/tn.jsonl 2>> $O/err.log || exit $?
  KGX_TN_SETS=6 timeout -k 10 120 python -u tools/exp_gemm_tn.py >> $O/tn.jsonl 2>> $O/err.log || exit $?
done
for R in 1 2; do
  timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_4.$R.json 2>> $O/err.log || exit $?
  KGX_TN_SETS=6 timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_6.$R.json 2>> $O/err.log || exit $?
done
