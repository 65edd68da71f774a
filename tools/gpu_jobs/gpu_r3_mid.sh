# Round 3: degree 3-7 rows of the 256 path in their own launch, prefetch depth 6 (main) vs 8 / 4 (variants).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/f256
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused256.py \
  > gpurun_out/f256/pytest_mid.log 2>&1 || { tail -40 gpurun_out/f256/pytest_mid.log; exit 1; }
tail -2 gpurun_out/f256/pytest_mid.log
: > gpurun_out/f256/ab_mid.log
for round in 0 1; do
  for lib in main mid8 mid4; do
    if [ $lib = main ]; then L=keras-geometric_amd/lib/libkgx.so; else L=keras-geometric_amd/lib/variants/libkgx_$lib.so; fi
    KGX_EXP_UNFUSED=0 KGX_LIB=$L timeout -k 10 240 python tools/exp_f256.py >> gpurun_out/f256/ab_mid.log 2>gpurun_out/f256/ab_$lib.err || exit $?
  done
done
cat gpurun_out/f256/ab_mid.log
