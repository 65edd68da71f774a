# round-2 checks: config-size parity tests, N>1 rehearsal through bench.py's own launcher, C4/C5 bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v -k "c4 or c5" --timeout 600 --timeout-method thread > gpurun_out/t3.log 2>&1 || exit $?
KGX_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --config c2 --steps 3 --warmup 1 > gpurun_out/reh.json 2> gpurun_out/reh.err || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/c4.json 2> gpurun_out/c4.err || exit $?
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit $?
