set -o pipefail
mkdir -p gpurun_out/calib
export TMPDIR=/tmp
timeout -k 10 400 python tools/exp_agg.py sweep > gpurun_out/sweep.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib/fetch -o run \
  --kernel-include-regex spmm -- python3 tools/exp_agg.py calib > gpurun_out/calib/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib/write -o run \
  --kernel-include-regex spmm -- python3 tools/exp_agg.py calib > gpurun_out/calib/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/calib/rdreq -o run \
  --kernel-include-regex spmm -- python3 tools/exp_agg.py calib > gpurun_out/calib/rdreq.log 2>&1 || true
