# Round 6: the NS hub fix-up on the head stream before the join (hidden behind the tail leg):
# fused / tiny / full-size / config tests, NS lines, kernel trace, FETCH / WRITE passes
# (-> pmc_ns.json, copied into profiles/r06 on the box) and the NS line as the driver runs it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6nsfix
mkdir -p $O profiles/r06
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_layers.py tests/test_gpu_tiny.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py \
  tests/test_gpu_kernels.py tests/test_gpu_backward.py > $O/pytest.log 2>&1 || exit $?
for R in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > $O/bench_ns.$R.json 2>> $O/err.log || exit $?
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_ns -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/trace_ns.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_ns -o run \
  --kernel-include-regex spmm -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold > $O/fetch_ns.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_ns -o run \
  --kernel-include-regex spmm -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold > $O/write_ns.log 2>&1 || exit $?
F=$(find $O/fetch_ns -name '*counter_collection.csv' | head -n 1)
W=$(find $O/write_ns -name '*counter_collection.csv' | head -n 1)
python tools/pmc_summary.py "$F" "$W" $O/pmc_ns.json --config ns || exit $?
cp $O/pmc_ns.json profiles/r06/pmc_ns.json
timeout -k 10 600 python -u bench.py > $O/bench_ns_final.json 2> $O/bench_ns_final.err || exit $?
timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/bench_train.json 2> $O/bench_train.err || exit $?
