# Round 5: NS fork mode 4 (main kernel with (den-1)/den of its grid, tails on the side stream in
# the slots left on every CU; KGX_SHARE_DEN 2 / 4 / 8) against the CU split (mode 3, default) -> gpurun_out/f4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/f4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiny.py -m gpu -q -k fork --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > $O/ns_split.$i.json 2>> $O/err.log || exit $?
  for d in 2 4 8; do
    KGX_FUSED_FORK=4 KGX_FUSED_CU_SPLIT=0 KGX_SHARE_DEN=$d timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > $O/ns_f4_den$d.$i.json 2>> $O/err.log || exit $?
  done
done
