set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_fused.json 2>/dev/null || exit $?
KGX_FUSED=0 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_unfused.json 2>/dev/null || exit $?
mkdir -p gpurun_out/prof_fused
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fused -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_fused/log 2>&1 || exit $?
