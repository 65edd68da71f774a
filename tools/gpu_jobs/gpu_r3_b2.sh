# round 3 batch 2: EXACT hub/fork A/B, tuned-unit NS sims, strong-config sims
set -o pipefail
mkdir -p gpurun_out/r3b2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "exact or hub or width" > gpurun_out/r3b2/pytest.log 2>&1 || exit $?
KGX_AB_WORK=exact timeout -k 10 600 python tools/exp_agg.py ab main main:KGX_EXACT_FORK=0 dyn32 main:KGX_HUB=0 > gpurun_out/r3b2/ab_exact.log 2>&1 || exit $?
bash tools/gpu_jobs/gpu_r3_sims.sh || exit $?
