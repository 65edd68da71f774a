# Round 5: the CU-split 256-wide launch (KGX_FUSED_CU_SPLIT): its GPU tests, then
# the C4 bench line with the split (model default) and without (KGX_F256_CU_SPLIT=0),
# two interleaved rounds -> gpurun_out/cus
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/cus
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused256.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/c4_split.$i.json 2> $O/c4_split.$i.err || exit $?
  KGX_F256_CU_SPLIT=0 timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/c4_nosplit.$i.json 2> $O/c4_nosplit.$i.err || exit $?
done
