# Round 6: C4 with KGX_F256_MID_TAIL = 200 by default -- the 256-wide GPU tests, the C4 kernel
# trace and PMC traffic (-> pmc_c4.json, copied into profiles/r06 on the box) and the C4 line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6c4f
mkdir -p $O profiles/r06
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused256.py tests/test_gpu_configs.py > $O/pytest.log 2>&1 || exit $?
bash tools/gpu_jobs/gpu_pmc_configs.sh c4 || exit $?
cp gpurun_out/prof/pmc_c4.json profiles/r06/pmc_c4.json
for R in 1 2; do
  timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 > $O/bench_c4.$R.json 2> $O/bench_c4.err || exit $?
done
