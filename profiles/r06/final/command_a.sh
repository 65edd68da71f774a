# Round 6 final measurement, part A (final sources): the whole GPU suite, smoke(), the NS
# kernel trace and FETCH_SIZE / WRITE_SIZE passes (-> pmc_ns.json, copied into profiles/r06 on
# the box so the bench line attaches it), the NS bench line as the driver runs it, and the NS
# training step with its kernel trace.  Outputs under gpurun_out/final.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O profiles/r06
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
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
timeout -k 10 600 python -u bench.py > $O/bench_ns.json 2> $O/bench_ns.err || exit $?
timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/bench_ns_train.json 2> $O/bench_ns_train.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_train -o run \
  -- python3 bench.py --train --steps 10 --warmup 2 > $O/trace_train.log 2>&1 || exit $?
