# Round 5: GPU suite + smoke + NS / C4 bench lines from the current sources -> gpurun_out/r5c
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench_ns.json 2> $O/bench_ns.err || exit $?
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
exit $rc
