# Round 3 close-out from the final sources: C4 rocprof stats + PMC (256 kernels changed last),
# the NS and C4 bench lines, then the whole GPU suite and smoke().
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/close
bash tools/gpu_jobs/gpu_pmc_configs.sh c4 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/close/bench_ns.json 2> gpurun_out/close/bench_ns.err || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cold > gpurun_out/close/bench_c4.json 2> gpurun_out/close/bench_c4.err || exit $?
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu \
  > gpurun_out/close/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/close/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/close/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
