# Round 3: item columns a tile ahead in the main 256 kernel: parity tests, then the C4 breakdown.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/f256
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused256.py \
  > gpurun_out/f256/pytest_icols.log 2>&1 || { tail -40 gpurun_out/f256/pytest_icols.log; exit 1; }
tail -3 gpurun_out/f256/pytest_icols.log
KGX_EXP_UNFUSED=0 timeout -k 10 240 python tools/exp_f256.py > gpurun_out/f256/ab_icols.log 2> gpurun_out/f256/ab_icols.err || exit $?
cat gpurun_out/f256/ab_icols.log
