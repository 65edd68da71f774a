# round 3: degree-1 tiny kernel with compact records and a second tile of gathers in flight
# (KGX_TINY1_DEPTH 2) -- GPU suite, exp_tiny check, A/B against the depth-1 build, then the N>1 rehearsal
set -o pipefail
mkdir -p gpurun_out/r3t1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3t1/pytest.log 2>&1 || { tail -40 gpurun_out/r3t1/pytest.log; exit 1; }
tail -3 gpurun_out/r3t1/pytest.log
timeout -k 10 300 python tools/exp_tiny.py > gpurun_out/r3t1/exp_tiny.log 2>&1 || { tail -20 gpurun_out/r3t1/exp_tiny.log; exit 1; }
cat gpurun_out/r3t1/exp_tiny.log
KGX_AB_WORK=both timeout -k 10 600 python tools/exp_agg.py ab main d1 > gpurun_out/r3t1/ab.log 2>&1 || { tail -20 gpurun_out/r3t1/ab.log; exit 1; }
tail -8 gpurun_out/r3t1/ab.log
bash tools/gpu_jobs/gpu_r3_rehearse.sh
