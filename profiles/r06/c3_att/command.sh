# Round 6 (A/B, the old library is a temporary build): GATv2 with the d att LDS reduction
# against the previous gatv2.hip (KGX_LIB=.../libkgx_oldgat.so): C3 line and C3 training step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c3ab
mkdir -p $O
OLD=$GRAFT_REPO_ROOT/keras-geometric_amd/lib/libkgx_oldgat.so
for R in 1 2 3; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-cold > $O/c3_new.$R.json 2>> $O/err.log || exit $?
  KGX_LIB=$OLD timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-cold > $O/c3_old.$R.json 2>> $O/err.log || exit $?
  timeout -k 10 300 python -u tools/bench_configs.py c3_train > $O/c3t_new.$R.json 2>> $O/err.log || exit $?
  KGX_LIB=$OLD timeout -k 10 300 python -u tools/bench_configs.py c3_train > $O/c3t_old.$R.json 2>> $O/err.log || exit $?
done
