# Round 3: fused-256 cost decomposition (debug builds: 1 no MFMA, 2 no stores, 3 neither, 4 gathers hit row 0).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/f256
: > gpurun_out/f256/dbg.log
for lib in main dbg1 dbg2 dbg3 dbg4; do
  if [ $lib = main ]; then L=keras-geometric_amd/lib/libkgx.so; else L=keras-geometric_amd/lib/variants/libkgx_$lib.so; fi
  KGX_EXP_UNFUSED=0 KGX_LIB=$L timeout -k 10 240 python tools/exp_f256.py >> gpurun_out/f256/dbg.log 2>gpurun_out/f256/dbg_$lib.err || exit $?
done
cat gpurun_out/f256/dbg.log
