# Round 3: 256 tail kernel wave order A/B (0 = half MFMA-first (main), 1 = all MFMA-first, 2 = all prepare-first).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/f256
: > gpurun_out/f256/ab_order.log
for round in 0 1; do
  for lib in main ord1 ord2; do
    if [ $lib = main ]; then L=keras-geometric_amd/lib/libkgx.so; else L=keras-geometric_amd/lib/variants/libkgx_$lib.so; fi
    KGX_EXP_UNFUSED=0 KGX_LIB=$L timeout -k 10 240 python tools/exp_f256.py >> gpurun_out/f256/ab_order.log 2>gpurun_out/f256/ab_$lib.err || exit $?
  done
done
cat gpurun_out/f256/ab_order.log
