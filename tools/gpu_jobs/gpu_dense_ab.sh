# kgx_dense A/B: GPU dense tests on the main library, then bench_dense.py per library, interleaved.
# usage: bash tools/gpu_jobs/gpu_dense_ab.sh variant1 [variant2 ...]   (main library always included)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dense_tests.log 2>&1 || exit $?
: > gpurun_out/dense_ab.log
for r in 0 1; do
  for v in main "$@"; do
    if [ "$v" = main ]; then lib=keras-geometric_amd/lib/libkgx.so; else lib=keras-geometric_amd/lib/variants/libkgx_$v.so; fi
    echo "round$r $v" >> gpurun_out/dense_ab.log
    KGX_LIB=$lib timeout -k 10 200 python tools/bench_dense.py --only ${ONLY:-C4,C5,NS} --reps 10 >> gpurun_out/dense_ab.log 2>&1 || exit $?
  done
done
