# Round 6: kgx_gemm_tn LDS form with and without the wave stagger (KGX_TN_STAGGER), register form.
# (KGX_TN_STAGGER was a temporary kernel variant, measured slower and removed; DESIGN.md §4 kgx_gemm_tn)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6tnst2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_gemm_tn.py > $O/pytest_st.log 2>&1 || exit $?
for R in 1 2; do
  timeout -k 10 120 python -u tools/exp_gemm_tn.py >> $O/tn.jsonl 2>> $O/err.log || exit $?
  KGX_TN_STAGGER=1 timeout -k 10 120 python -u tools/exp_gemm_tn.py >> $O/tn.jsonl 2>> $O/err.log || exit $?
  KGX_TN_LDS=0 timeout -k 10 120 python -u tools/exp_gemm_tn.py >> $O/tn.jsonl 2>> $O/err.log || exit $?
done
