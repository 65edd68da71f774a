# Round 3: double-buffered 256 tail kernel (default build) vs the single-buffer one (variant tiny1).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/f256
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused256.py \
  > gpurun_out/f256/pytest_tiny2.log 2>&1 || { tail -40 gpurun_out/f256/pytest_tiny2.log; exit 1; }
tail -3 gpurun_out/f256/pytest_tiny2.log
: > gpurun_out/f256/ab_tiny2.log
for round in 0 1; do
  for lib in main tiny1; do
    if [ $lib = main ]; then L=keras-geometric_amd/lib/libkgx.so; else L=keras-geometric_amd/lib/variants/libkgx_$lib.so; fi
    KGX_EXP_UNFUSED=0 KGX_LIB=$L timeout -k 10 240 python tools/exp_f256.py >> gpurun_out/f256/ab_tiny2.log 2>gpurun_out/f256/ab_$lib.err || exit $?
  done
done
cat gpurun_out/f256/ab_tiny2.log
