# Round-4 C4 refresh after the 256-wide kernels' root-row prefetch (spmm_gemm256.hip):
# the GPU tests that run those kernels, the C4 PMC passes and kernel stats, and the
# C4 bench line with the PMC traffic attached.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final gpurun_out/prof
O=gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  -k "256 or c4 or gin or GIN or sharded" > $O/pytest_c4.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_c4.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_jobs/gpu_pmc_configs.sh c4 || exit $?
cp gpurun_out/prof/pmc_c4.json profiles/r04/pmc_c4.json || exit 1
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 > $O/bench_line_c4.json 2> $O/bench_line_c4.err || exit $?
