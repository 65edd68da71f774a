# Round 5 (measured, not kept: tools/experiments/round5_exact_cu_split.patch): EXACT aggregation
# (KGX_EXACT_CU_SPLIT=8, read once per process): the EXACT / bit-identity GPU tests under it, then
# NS --exact bench lines with and without, interleaved -> gpurun_out/exs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/exs
mkdir -p $O
KGX_EXACT_CU_SPLIT=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py -m gpu -q -k "exact or bit or fullsize" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --exact --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/exact_nosplit.$i.json 2>> $O/err.log || exit $?
  KGX_EXACT_CU_SPLIT=8 timeout -k 10 200 python bench.py --exact --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/exact_split.$i.json 2>> $O/err.log || exit $?
done
