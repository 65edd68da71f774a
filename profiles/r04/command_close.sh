# Round-4 close-out from the final sources (one gpurun call), after the fused
# kernels' split refactor (spmm_gemm.hip, spmm_gemm256.hip changed, so NS's and
# C4's PMC summaries are re-measured; C3 / C5 sources are unchanged): the GPU
# suite, smoke(), NS and C4 kernel stats + FETCH_SIZE / WRITE_SIZE passes (copied
# into profiles/r04/ on the box, where bench.py's pmc_traffic finds them), then
# the bench lines (NS with the CPU baseline, C3, C4, C5, NS EXACT).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/close gpurun_out/prof
O=gpurun_out/close
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  > $O/pytest_gpu_final.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu_final.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof/trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o run \
  --kernel-include-regex spmm -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o run \
  --kernel-include-regex spmm -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/write.log 2>&1 || exit $?
F=$(find gpurun_out/prof/fetch -name '*counter_collection.csv' | head -n 1)
W=$(find gpurun_out/prof/write -name '*counter_collection.csv' | head -n 1)
python tools/pmc_summary.py "$F" "$W" gpurun_out/prof/pmc_ns.json --config ns || exit $?
cp gpurun_out/prof/pmc_ns.json profiles/r04/pmc_ns.json || exit 1
bash tools/gpu_jobs/gpu_pmc_configs.sh c4 || exit $?
cp gpurun_out/prof/pmc_c4.json profiles/r04/pmc_c4.json || exit 1
timeout -k 10 900 python bench.py --steps 20 --warmup 3 > $O/bench_line_ns.json 2> $O/bench_line_ns.err || exit $?
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 > $O/bench_line_$c.json 2> $O/bench_line_$c.err || exit $?
done
timeout -k 10 300 python bench.py --exact --steps 20 --warmup 3 --no-cpu-baseline --no-cold > $O/bench_line_exact.json 2> $O/bench_line_exact.err || exit $?
