# rocprofv3 kernel stats + PMC traffic (FETCH_SIZE, WRITE_SIZE; separate passes) for
# the dominant kernels of C3 (gatv2_kernel), C4 (spmm_kernel F256, dense_kernel 256->256)
# and C5 (spmm_kernel F100, dense_kernel (100+100)->100).  Usage: bash tools/gpu_jobs/gpu_pmc_configs.sh c3 c4 c5
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for c in "$@"; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/prof/bench_$c.json 2> gpurun_out/prof/bench_$c.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace_$c -o run \
    -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/prof/trace_$c.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch_$c -o run \
    --kernel-include-regex 'spmm|gatv2|dense' -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/prof/fetch_$c.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write_$c -o run \
    --kernel-include-regex 'spmm|gatv2|dense' -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/prof/write_$c.log 2>&1 || exit $?
  F=$(find gpurun_out/prof/fetch_$c -name '*counter_collection.csv' | head -n 1)
  W=$(find gpurun_out/prof/write_$c -name '*counter_collection.csv' | head -n 1)
  python tools/pmc_summary.py "$F" "$W" gpurun_out/prof/pmc_$c.json --config $c || exit $?
done
