# Round 5: NS training step and C3 training step with the CU split (default rule) and without
# (KGX_FUSED_CU_SPLIT=0), two interleaved rounds -> gpurun_out/r5tr
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5tr
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python tools/bench_configs.py ns_train > $O/ns_train_split.$i.json 2>> $O/err.log || exit $?
  KGX_FUSED_CU_SPLIT=0 timeout -k 10 300 python tools/bench_configs.py ns_train > $O/ns_train_nosplit.$i.json 2>> $O/err.log || exit $?
done
