# Tiny-tail fused kernel: its own tests, the fused-path tests, then the NS bench.
set -o pipefail
mkdir -p gpurun_out/tiny
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tiny.py \
  tests/test_gpu_configs.py tests/test_gpu_kernels.py tests/test_gpu_layers.py tests/test_gpu_fullsize.py \
  tests/test_gpu_distributed.py tests/test_gpu_backward.py > gpurun_out/tiny/tests.log 2>&1 || { tail -40 gpurun_out/tiny/tests.log; exit 1; }
tail -2 gpurun_out/tiny/tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/tiny/bench_ns.json 2> gpurun_out/tiny/bench_ns.err || exit $?
cat gpurun_out/tiny/bench_ns.json
