# round 3: cost decomposition of the degree <= 2 tiny kernels on the NS layer (experiment build,
# KGX_FUSED_DEBUG 4 no MFMA, 8 no stores, 12 neither, 16 gathers all from row 0); rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out/r3dec
export TMPDIR=/tmp
LIB=$PWD/keras-geometric_amd/lib/variants/libkgx_exp.so
for dbg in 0 4 8 12 16 0; do
  KGX_LIB=$LIB KGX_FUSED_DEBUG=$dbg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3dec/d$dbg -o run \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/r3dec/d$dbg.json 2> gpurun_out/r3dec/d$dbg.err || exit $?
  f=$(find gpurun_out/r3dec/d$dbg -name '*kernel_stats.csv' | head -n 1)
  echo "== debug $dbg: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3dec/d$dbg.json)"
  python3 - "$f" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    if 'spmm_gemm' in row['Name']:
        print(f"  {row['Name'][30:95]:65s} avg {float(row['AverageNs'])/1e6:.3f} ms")
PY
done
