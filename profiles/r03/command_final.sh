# Final profiles for the current sources: NS (bench + rocprof stats + PMC), C3/C4/C5
# (rocprof + PMC), then the bench lines with the fresh PMC traffic attached.
set -o pipefail
bash profiles/r03/command_ns.sh || exit $?
bash tools/gpu_jobs/gpu_pmc_configs.sh c3 c4 c5 || exit $?
cp gpurun_out/prof/pmc_ns.json gpurun_out/prof/pmc_c3.json gpurun_out/prof/pmc_c4.json gpurun_out/prof/pmc_c5.json profiles/r03/ || exit 1
bash tools/gpu_jobs/gpu_bench_lines.sh || exit $?
EXACT=1 timeout -k 10 300 python bench.py --exact --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/lines/bench_exact.json 2> gpurun_out/lines/bench_exact.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace_exact -o run \
  -- python3 bench.py --exact --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/prof/trace_exact.log 2>&1 || exit $?
