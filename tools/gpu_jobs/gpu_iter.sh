# quick iteration: selected GPU tests + fused/unfused NS bench (no CPU baseline)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_fused.json 2>/dev/null || exit $?
KGX_FUSED=0 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_unfused.json 2>/dev/null || exit $?
