# Round 3: 256 kernels with the packed-pair split (split3_pair_rn) in put_row: parity tests + C4 breakdown.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/f256
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused256.py \
  > gpurun_out/f256/pytest_split.log 2>&1 || { tail -40 gpurun_out/f256/pytest_split.log; exit 1; }
tail -3 gpurun_out/f256/pytest_split.log
: > gpurun_out/f256/ab_split.log
for round in 0 1; do
  KGX_EXP_UNFUSED=0 timeout -k 10 240 python tools/exp_f256.py >> gpurun_out/f256/ab_split.log 2>gpurun_out/f256/ab_split.err || exit $?
done
cat gpurun_out/f256/ab_split.log
