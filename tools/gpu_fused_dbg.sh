set -o pipefail
export TMPDIR=/tmp
KGX_FUSED_DEBUG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/fdbg1.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/fdbg0.json 2>/dev/null || exit $?
