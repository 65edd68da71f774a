# Round 3: the 256-wide fused kernel (GINConv C4): parity tests, C4 bench fused vs unfused, rocprof stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/f256
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused256.py \
  > gpurun_out/f256/pytest.log 2>&1 || { tail -40 gpurun_out/f256/pytest.log; exit 1; }
tail -3 gpurun_out/f256/pytest.log
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cold > gpurun_out/f256/bench_c4.json 2> gpurun_out/f256/bench_c4.err || exit $?
KGX_FUSED256=0 timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cold --no-cpu-baseline > gpurun_out/f256/bench_c4_unfused.json 2> gpurun_out/f256/bench_c4_unfused.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f256/trace_c4 -o run \
  -- python3 bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/f256/trace_c4.log 2>&1 || exit $?
cat gpurun_out/f256/bench_c4.json gpurun_out/f256/bench_c4_unfused.json
find gpurun_out/f256/trace_c4 -name '*kernel_stats.csv' -exec cat {} \;
