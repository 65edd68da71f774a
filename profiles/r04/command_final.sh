# Round-4 final run from the final sources (one gpurun call): the GPU suite,
# smoke(), C5's PMC passes again (spmm.hip changed after profiles/r04/command_pmc.sh),
# then the bench lines with the PMC traffic attached (NS with the CPU baseline,
# C3, C4, C5, NS EXACT) and the EXACT kernel stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final gpurun_out/prof
O=gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  > $O/pytest_gpu_final.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu_final.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
bash tools/gpu_jobs/gpu_pmc_configs.sh c5 || exit $?
cp gpurun_out/prof/pmc_c5.json profiles/r04/pmc_c5.json || exit 1
timeout -k 10 900 python bench.py --steps 20 --warmup 3 > $O/bench_line_ns.json 2> $O/bench_line_ns.err || exit $?
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 > $O/bench_line_$c.json 2> $O/bench_line_$c.err || exit $?
done
timeout -k 10 300 python bench.py --exact --steps 20 --warmup 3 --no-cpu-baseline --no-cold > $O/bench_line_exact.json 2> $O/bench_line_exact.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_exact -o run \
  -- python3 bench.py --exact --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/trace_exact.log 2>&1
