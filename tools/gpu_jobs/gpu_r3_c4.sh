# Round 3: C4 with the fused 256 kernels by default: full-size C4 tests, bench line, rocprof stats + PMC.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_fused256.py \
  "tests/test_gpu_configs.py::test_c4_gin_linearity_and_mlp" "tests/test_gpu_configs.py::test_c4_gin_csr_and_exact_rows" \
  > gpurun_out/c4/pytest.log 2>&1 || { tail -40 gpurun_out/c4/pytest.log; exit 1; }
tail -3 gpurun_out/c4/pytest.log
bash tools/gpu_jobs/gpu_pmc_configs.sh c4 || exit $?
cat gpurun_out/prof/bench_c4.json
