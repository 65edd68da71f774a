# Round 6: C4 KGX_F256_MID_TAIL around 200 per mille (interleaved, three rounds) and a kernel
# trace at 200.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6bal2
mkdir -p $O
for R in 1 2 3; do
  for V in 0 150 200 250; do
    KGX_F256_MID_TAIL=$V timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-cold \
      | sed "s/^/{\"mid_tail\": $V, \"line\": /; s/\$/}/" >> $O/c4.jsonl 2>> $O/err.log || exit $?
  done
done
cd /tmp && KGX_F256_MID_TAIL=200 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace_c4 -o run \
  -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $GRAFT_REPO_ROOT/$O/trace_c4.log 2>&1 || exit $?
