# Round 6: the NS EXACT (bit-identical aggregation) line on the final sources.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6exact
mkdir -p $O
for R in 1 2; do
  timeout -k 10 300 python -u bench.py --exact --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_exact.$R.json 2>> $O/err.log || exit $?
done
