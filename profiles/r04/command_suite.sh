# Round-4 close-out: the whole GPU suite and smoke() from the final sources.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
O=gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  > $O/pytest_gpu_final.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu_final.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
