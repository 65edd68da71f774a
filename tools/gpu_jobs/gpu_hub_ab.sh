# Hub-kernel variants: synthetic hub graphs (tools/exp_hub_synth.py) and the
# NS EXACT aggregation (tools/exp_hub.py) per library.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/hubab
for v in "$@"; do
  if [ "$v" = main ]; then lib=$PWD/keras-geometric_amd/lib/libkgx.so; else lib=$PWD/keras-geometric_amd/lib/variants/libkgx_$v.so; fi
  echo "== $v" >> gpurun_out/hubab/synth.log
  KGX_LIB=$lib timeout -k 10 240 python3 tools/exp_hub_synth.py >> gpurun_out/hubab/synth.log 2>&1 || exit 1
  KGX_LIB=$lib timeout -k 10 240 python3 tools/exp_hub.py >> gpurun_out/hubab/synth.log 2>&1 || exit 1
done
cat gpurun_out/hubab/synth.log
