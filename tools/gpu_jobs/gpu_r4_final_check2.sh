#!/bin/bash
# Round 4, after the pull-plan change in distributed.py: the GPU suite (incl.
# the threaded-rank sharded tests) and smoke() from the final tree.
set -o pipefail
mkdir -p gpurun_out/r4fc2 && rm -f gpurun_out/r4fc2/*
export TMPDIR=/tmp
O=gpurun_out/r4fc2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
