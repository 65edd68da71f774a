# Round 6: the driver's own round-end commands on the final tree: smoke(), the default bench line
# (N = 1, as the driver runs it) and the training line with its traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final_f
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench_ns.json 2> $O/bench_ns.err || exit $?
timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/bench_ns_train.json 2> $O/bench_ns_train.err || exit $?
