# Round 3 (final C4 kernels): full-size C4 tests, C4 rocprof stats + PMC + bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_fused256.py \
  "tests/test_gpu_configs.py::test_c4_gin_linearity_and_mlp" > gpurun_out/c4/pytest.log 2>&1 || { tail -40 gpurun_out/c4/pytest.log; exit 1; }
tail -3 gpurun_out/c4/pytest.log
bash tools/gpu_jobs/gpu_pmc_configs.sh c4 || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cold > gpurun_out/c4/bench_line_c4.json 2> gpurun_out/c4/bench_line_c4.err || exit $?
cat gpurun_out/c4/bench_line_c4.json
