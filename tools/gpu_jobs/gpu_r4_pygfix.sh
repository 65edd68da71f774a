#!/bin/bash
# Round 4: the HIP GCN / GATv2 / GIN layers on the reference tests' PyG-comparison
# fixtures against the PyG restatement, at those tests' tolerances.
set -o pipefail
mkdir -p gpurun_out/r4pf
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pyg_fixtures.py -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/r4pf/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4pf/pytest.log
exit $rc
