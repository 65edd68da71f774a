# round 3: D^T direct stores in the main (spmm_gemm_kernel) and short-row fused kernels vs their LDS out-tile
# forms (fts0 / sts0 builds): fused-op GPU tests, then NS bench under rocprof, interleaved twice
set -o pipefail
mkdir -p gpurun_out/r3ts2
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_layers.py tests/test_gpu_kernels.py tests/test_gpu_fullsize.py \
  tests/test_gpu_distributed.py tests/test_gpu_backward.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3ts2/pytest.log 2>&1 \
  || { tail -30 gpurun_out/r3ts2/pytest.log; exit 1; }
tail -2 gpurun_out/r3ts2/pytest.log
for r in 1 2; do
  for v in main fts0 sts0; do
    lib=$PWD/keras-geometric_amd/lib/libkgx.so; [ $v = main ] || lib=$PWD/keras-geometric_amd/lib/variants/libkgx_$v.so
    KGX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3ts2/${v}_$r -o run \
      -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/r3ts2/${v}_$r.json 2> gpurun_out/r3ts2/${v}_$r.err || exit $?
    f=$(find gpurun_out/r3ts2/${v}_$r -name '*kernel_stats.csv' | head -n 1)
    echo "== $v round $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3ts2/${v}_$r.json)"
    python3 - "$f" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    if 'spmm_gemm' in row['Name']:
        print(f"  {row['Name'][30:95]:65s} avg {float(row['AverageNs'])/1e6:.3f} ms")
PY
  done
done
