# Round 5: NS fused op with the main kernel and the short + tiny launches on
# disjoint CU sets (KGX_FUSED_FORK=3) against the one-stream order, interleaved
# bench lines; the fork bit-identity tests; a rocprofv3 kernel trace of C4 (the
# CU-masked streams' exit under the profiler) -> gpurun_out/nsc
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/nsc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiny.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k fork > $O/pytest.log 2>&1 || exit $?
for i in 1 2 3; do
  for f in 0 3; do
    KGX_FUSED_FORK=$f timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold \
      > $O/ns_fork$f.$i.json 2> $O/ns_fork$f.$i.err || exit $?
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o run \
  -- python3 bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline --no-cold > $O/trace_c4.log 2>&1
echo "rocprofv3 c4 rc $?" >> $O/pytest.log
