set -o pipefail
export TMPDIR=/tmp
for h in 0 1 2 3; do
  KGX_SPMM_HINTS=$h timeout -k 10 200 python tools/exp_agg.py ns >> gpurun_out/hints.log 2>/dev/null || exit $?
done
mkdir -p gpurun_out/hit
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/hit/h0 -o run \
  --kernel-include-regex spmm_kernel -- python3 tools/exp_agg.py ns > gpurun_out/hit/h0.log 2>&1 || exit $?
