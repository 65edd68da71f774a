# kgx_dense A/B by environment (same library): dense tests, then bench_dense.py per setting, interleaved.
# usage: bash tools/gpu_jobs/gpu_dense_env_ab.sh "KGX_DENSE_CSTORE=1" ...   (the plain environment always included)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_layers.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dense_tests.log 2>&1 || exit $?
: > gpurun_out/dense_env_ab.log
for r in 0 1; do
  for e in "" "$@"; do
    echo "round$r [$e]" >> gpurun_out/dense_env_ab.log
    env $e timeout -k 10 200 python tools/bench_dense.py --only ${ONLY:-C4,C5,NS,C3} --reps 10 >> gpurun_out/dense_env_ab.log 2>&1 || exit $?
  done
done
