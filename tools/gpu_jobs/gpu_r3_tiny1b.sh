# round 3: bisect the compact-record degree-1 tiny kernel on the NS graph (depth 2 vs depth 1 build),
# then the tiny GPU tests (which now assert the records are read)
set -o pipefail
mkdir -p gpurun_out/r3t1b
export TMPDIR=/tmp
timeout -k 10 300 python tools/exp_tiny.py > gpurun_out/r3t1b/exp_tiny_main.log 2>&1; rc=$?; echo "main rc=$rc"; [ $rc -le 1 ] || exit $rc
cat gpurun_out/r3t1b/exp_tiny_main.log | grep -v amdgpu.ids
KGX_LIB=$PWD/keras-geometric_amd/lib/variants/libkgx_d1.so timeout -k 10 300 python tools/exp_tiny.py \
  > gpurun_out/r3t1b/exp_tiny_d1.log 2>&1; rc=$?; echo "d1 rc=$rc"; [ $rc -le 1 ] || exit $rc
cat gpurun_out/r3t1b/exp_tiny_d1.log | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiny.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3t1b/pytest.log 2>&1; echo "pytest rc=$?"
tail -30 gpurun_out/r3t1b/pytest.log
