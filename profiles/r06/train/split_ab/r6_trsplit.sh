# Round 6: the NS training step with the dx pass CU-split (default) or one-stream (KGX_FUSED_CU_SPLIT=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6trsplit
mkdir -p $O
for R in 1 2 3; do
  timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_split.$R.json 2>> $O/err.log || exit $?
  KGX_FUSED_CU_SPLIT=0 timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_nosplit.$R.json 2>> $O/err.log || exit $?
done
