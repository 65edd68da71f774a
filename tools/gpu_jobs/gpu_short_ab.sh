# Short-row fused kernel: variants / debug decomposition (tools/exp_short.py).
# usage: bash tools/gpu_jobs/gpu_short_ab.sh lib[:DEBUG] ...
set -o pipefail
mkdir -p gpurun_out
for spec in "$@"; do
  v=${spec%%:*}; d=${spec#*:}; [ "$d" = "$spec" ] && d=0
  if [ "$v" = main ]; then lib=$PWD/keras-geometric_amd/lib/libkgx.so; else lib=$PWD/keras-geometric_amd/lib/variants/libkgx_$v.so; fi
  KGX_LIB=$lib KGX_FUSED_DEBUG=$d timeout -k 10 200 python3 tools/exp_short.py 2>&1 | grep short_ms | tee -a gpurun_out/short_ab.log || exit 1
done
