# round 3: the new parity tests (GATv2 kink, GATv2 layer backward, sharded C4 / C5 at full size)
set -o pipefail
mkdir -p gpurun_out/r3tests
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gatv2_conditioning.py "tests/test_gpu_backward.py::test_gatv2_layer_backward" \
  > gpurun_out/r3tests/gatv2.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu -s \
  ${SHARD_K:+-k "$SHARD_K"} tests/test_gpu_sharded_fullsize.py > gpurun_out/r3tests/sharded.log 2>&1 || exit $?
