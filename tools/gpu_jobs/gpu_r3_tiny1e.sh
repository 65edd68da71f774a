# round 3: degree-1 tiny kernel, final form (compact records, rows g + 16 j, two tiles of gathers in flight,
# 32-bit scalar tile indices): tiny GPU tests, the full-size bit-identity test, exp_tiny timing, NS bench
set -o pipefail
mkdir -p gpurun_out/r3t1e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py "tests/test_gpu_fullsize.py::test_tiny_tail_bit_identical_fullsize" \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/r3t1e/pytest.log 2>&1 || { tail -30 gpurun_out/r3t1e/pytest.log; exit 1; }
tail -2 gpurun_out/r3t1e/pytest.log
timeout -k 10 400 python tools/exp_tiny.py > gpurun_out/r3t1e/exp_tiny.log 2>&1 || { tail -20 gpurun_out/r3t1e/exp_tiny.log; exit 1; }
grep -E '^\{' gpurun_out/r3t1e/exp_tiny.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3t1e/bench_ns.json 2> gpurun_out/r3t1e/bench_ns.err || { tail -20 gpurun_out/r3t1e/bench_ns.err; exit 1; }
cut -c1-400 gpurun_out/r3t1e/bench_ns.json
