# Round 6 closing check on the final sources: the whole GPU suite, smoke(), every bench line
# (NS as the driver runs it, C3 / C4 / C5 with their PMC traffic, the training step).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final_d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench_ns.json 2> $O/bench_ns.err || exit $?
for c in c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
done
timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/bench_ns_train.json 2> $O/bench_ns_train.err || exit $?
