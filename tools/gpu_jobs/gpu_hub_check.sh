# EXACT hub-row kernel: bitwise tests, then the EXACT bench under rocprofv3.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ex
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_configs.py -k "exact or hub or saturates or widths or nan" \
  > gpurun_out/ex/tests.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py -k "exact" >> gpurun_out/ex/tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ex/trace -o run -- python3 bench.py --exact --steps 5 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/ex/bench.json 2> gpurun_out/ex/bench.err &&
timeout -k 10 200 python tools/exp_hub.py > gpurun_out/ex/hub.json 2>&1
rc=$?
tail -5 gpurun_out/ex/tests.log
exit $rc
