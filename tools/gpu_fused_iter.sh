set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 -k "fused or gcn" > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_fused.json 2>/dev/null || exit $?
