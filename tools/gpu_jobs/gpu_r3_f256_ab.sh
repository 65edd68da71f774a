# Round 3: fused-256 kernel by part (long / short) for the main build and block-size variants, then the
# full GPU suite and the NS profile (bench + rocprofv3 stats + PMC).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/f256
: > gpurun_out/f256/ab.log
for lib in main u6 u8; do
  if [ $lib = main ]; then L=keras-geometric_amd/lib/libkgx.so; else L=keras-geometric_amd/lib/variants/libkgx_$lib.so; fi
  KGX_EXP_UNFUSED=$([ $lib = main ] && echo 1 || echo 0) KGX_LIB=$L timeout -k 10 240 python tools/exp_f256.py >> gpurun_out/f256/ab.log 2>gpurun_out/f256/ab_$lib.err || exit $?
done
cat gpurun_out/f256/ab.log
bash tools/gpu_jobs/gpu_r3_suite_ns.sh || exit $?
