# Round 6: balancing the CU-split legs -- NS: the first KGX_FUSED_SHORT_HEAD / 1000 of the short
# rows on the head's 192 CUs after the main kernel; C4: the last KGX_F256_MID_TAIL / 1000 of the
# degree 3..7 rows on the tail's 64 CUs after the degree <= 2 tail.  Bit-identity tests, then
# interleaved bench sweeps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6bal
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused256.py -k "cu_split" "tests/test_gpu_layers.py::test_hip_graph_capture_cu_split" > $O/pytest.log 2>&1 || exit $?
for R in 1 2; do
  for V in 0 40 80 150; do
    KGX_FUSED_SHORT_HEAD=$V timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold \
      | sed "s/^/{\"short_head\": $V, \"line\": /; s/\$/}/" >> $O/ns.jsonl 2>> $O/err.log || exit $?
  done
  for V in 0 100 200 300; do
    KGX_F256_MID_TAIL=$V timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-cold \
      | sed "s/^/{\"mid_tail\": $V, \"line\": /; s/\$/}/" >> $O/c4.jsonl 2>> $O/err.log || exit $?
  done
done
