# Round 5 (measured, not kept: tools/experiments/round5_f256_mid_after.patch): C4 with the degree 3..7 launch after the CU split's join on the whole GPU
# (KGX_F256_MID_AFTER=1) against after the long rows on the head's 192 CUs: the 256-wide
# bit-identity tests with it on, then C4 bench lines interleaved -> gpurun_out/mid
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/mid
mkdir -p $O
KGX_F256_MID_AFTER=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fused256.py tests/test_gpu_layers.py -m gpu -q -k "cu_split or fused256" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/c4_off.$i.json 2>> $O/err.log || exit $?
  KGX_F256_MID_AFTER=1 timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/c4_on.$i.json 2>> $O/err.log || exit $?
done
