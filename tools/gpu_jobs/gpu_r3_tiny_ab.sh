# round 3: NS fused op A/B of the tiny-row kernel's rows per group (degree-1 tail)
set -o pipefail
mkdir -p gpurun_out/r3tiny
export TMPDIR=/tmp
KGX_AB_WORK=both timeout -k 10 900 python tools/exp_agg.py ab main t5 t6 > gpurun_out/r3tiny/ab.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3tiny/prof -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/r3tiny/prof.log 2>&1 || exit $?
