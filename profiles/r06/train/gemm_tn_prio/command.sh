# Round 6 (experiment build): kgx_gemm_tn warp-specialised form with producer waves at raised
# issue priority (KGX_TN_PRIO=1) or consumer waves (2) against equal priority (0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6tnprio
mkdir -p $O
for R in 1 2 3; do
  for P in 0 1 2; do
    KGX_TN_PRIO=$P timeout -k 10 120 python -u tools/exp_gemm_tn.py >> $O/tn.jsonl 2>> $O/err.log || exit $?
  done
done
