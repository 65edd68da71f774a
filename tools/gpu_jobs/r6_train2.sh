# Round 6: kgx_gemm_tn with float4 loads + two steps of prefetch: its tests, the NS training
# step with kernel stats, then the C5 row-width sweep (tools/gpu_jobs/r6_c5sector.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6t2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_gemm_tn.py tests/test_gpu_backward.py > $O/pytest.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_train -o train \
  -- python -u $GRAFT_REPO_ROOT/bench.py --train --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/$O/bench_ns_train.json 2> $GRAFT_REPO_ROOT/$O/prof_train.err || exit $?
cd "$GRAFT_REPO_ROOT" && bash tools/gpu_jobs/r6_c5sector.sh
