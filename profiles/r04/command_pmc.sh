# Round-4 profiles from the final sources (one gpurun call): NS (bench line +
# rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes -> pmc_ns.json) and the
# C3 / C4 / C5 configs (tools/gpu_jobs/gpu_pmc_configs.sh).  The pmc_*.json files
# are then committed under profiles/r04/, where bench.py's pmc_traffic finds them.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 python bench.py --steps 20 --warmup 3 > gpurun_out/prof/bench_ns.json 2> gpurun_out/prof/bench_ns.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof/trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o run \
  --kernel-include-regex spmm -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o run \
  --kernel-include-regex spmm -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/write.log 2>&1 || exit $?
F=$(find gpurun_out/prof/fetch -name '*counter_collection.csv' | head -n 1)
W=$(find gpurun_out/prof/write -name '*counter_collection.csv' | head -n 1)
python tools/pmc_summary.py "$F" "$W" gpurun_out/prof/pmc_ns.json --config ns || exit $?
bash tools/gpu_jobs/gpu_pmc_configs.sh c3 c4 c5
