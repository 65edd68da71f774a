# Round-3 final profiles for the current sources (one gpurun call each part):
#   NS: bash profiles/r03/command_ns.sh  (bench + rocprofv3 stats + PMC; run earlier, same spmm_gemm.hip)
#   C4: bash tools/gpu_jobs/gpu_pmc_configs.sh c4   (fused 256 kernels)
# This script: C3 / C5 rocprof + PMC, the bench lines (PMC traffic attached from profiles/r03), EXACT.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_jobs/gpu_pmc_configs.sh c3 c5 || exit $?
cp gpurun_out/prof/pmc_c3.json gpurun_out/prof/pmc_c5.json profiles/r03/ || exit 1
bash tools/gpu_jobs/gpu_bench_lines.sh || exit $?
mkdir -p gpurun_out/lines
timeout -k 10 300 python bench.py --exact --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/lines/bench_exact.json 2> gpurun_out/lines/bench_exact.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace_exact -o run \
  -- python3 bench.py --exact --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/prof/trace_exact.log 2>&1 || exit $?
