# round 3: degree-1 tiny kernel bad rows -- which change causes them: the row map / vector record loads
# (strided build), loads in flight across the hand-off barrier (sync build), or the pipeline depth (d1 build)
set -o pipefail
mkdir -p gpurun_out/r3t1d
export TMPDIR=/tmp
for v in main strided sync; do
  lib=keras-geometric_amd/lib/libkgx.so
  [ $v = main ] || lib=keras-geometric_amd/lib/variants/libkgx_$v.so
  KGX_LIB=$PWD/$lib timeout -k 10 400 python tools/exp_tiny.py > gpurun_out/r3t1d/$v.log 2>&1; rc=$?
  echo "$v rc=$rc"; [ $rc -le 1 ] || exit $rc
  grep -E '^\{' gpurun_out/r3t1d/$v.log | cut -c1-400
done
