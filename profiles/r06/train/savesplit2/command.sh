# Round 6: with the backward's dx pass one-stream, the training forward (P kept) CU-split
# (KGX_SAVE_CU_SPLIT=1, a temporary ops.py switch, not in the tree) against one-stream (default).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ss2
mkdir -p $O
for R in 1 2 3; do
  timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_default.$R.json 2>> $O/err.log || exit $?
  KGX_SAVE_CU_SPLIT=1 timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_savesplit.$R.json 2>> $O/err.log || exit $?
done
