# Round 5: C4 tail interleave A/B: shipped / one-block period (KGX_T2_ILV=1) /
# fenced per-k-step pieces (KGX_T2_ILV=3); out_bits must match the shipped build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/t2i
mkdir -p $O
: > $O/ab.log
for round in 0 1; do
  for lib in main t2i1 t2i3; do
    if [ $lib = main ]; then L=keras-geometric_amd/lib/libkgx.so; else L=keras-geometric_amd/lib/variants/libkgx_$lib.so; fi
    KGX_EXP_UNFUSED=0 KGX_LIB=$L timeout -k 10 240 python tools/exp_f256.py >> $O/ab.log 2> $O/$lib.err || exit $?
  done
done
