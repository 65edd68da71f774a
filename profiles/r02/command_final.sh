# Final profiles for the current sources: NS (bench + rocprof stats + PMC), C3/C4/C5
# (rocprof + PMC), then the bench lines with the fresh PMC traffic attached.
set -o pipefail
bash profiles/r02/command_ns.sh || exit $?
bash tools/gpu_jobs/gpu_pmc_configs.sh c3 c4 c5 || exit $?
cp gpurun_out/prof/pmc_ns.json gpurun_out/prof/pmc_c3.json gpurun_out/prof/pmc_c4.json gpurun_out/prof/pmc_c5.json profiles/r02/ || exit 1
bash tools/gpu_jobs/gpu_bench_lines.sh || exit $?
EXACT=1 timeout -k 10 300 python bench.py --exact --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/lines/bench_exact.json 2> gpurun_out/lines/bench_exact.err || exit $?
