# Round 6: the CU split's masks checked on the hardware (kgx_cu_split_census).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6census
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cu_census.py > $O/pytest.log 2>&1 || exit $?
