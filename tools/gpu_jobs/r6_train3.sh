# Round 6: the NS training step, serial dW (the default now), with the forward-with-P launch
# (KGX_SAVE_CU_SPLIT was a temporary ops.py switch, not in the tree; result in DESIGN.md, verdict item 7)
# CU-split (KGX_SAVE_CU_SPLIT=1) or not, and a kernel trace of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6train3
mkdir -p $O
for R in 1 2; do
  timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_def.$R.json 2>> $O/train.err || exit $?
  KGX_SAVE_CU_SPLIT=1 timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/train_savesplit.$R.json 2>> $O/train.err || exit $?
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o train \
  -- python -u $GRAFT_REPO_ROOT/bench.py --train --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof_train.json 2> $GRAFT_REPO_ROOT/$O/prof.err || exit $?
