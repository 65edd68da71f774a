# round 3 batch 3: EXACT hub dynamic A/B + tuned-unit NS sims
set -o pipefail
mkdir -p gpurun_out/r3b3
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_configs.py -k "exact or hub or width or c2" > gpurun_out/r3b3/pytest.log 2>&1 || exit $?
KGX_AB_WORK=exact timeout -k 10 600 python tools/exp_agg.py ab main main:KGX_EXACT_DYN=0 > gpurun_out/r3b3/ab_exact.log 2>&1 || exit $?
: > gpurun_out/r3b3/sim_ns.jsonl
for L in 0 400; do
  timeout -k 10 600 python tools/shard_sim.py --config ns --world 8 --merged 1 --merge-unit step,chunk,none \
    --chunks 1,2 --link-gbps $L --steps 5 >> gpurun_out/r3b3/sim_ns.jsonl 2>> gpurun_out/r3b3/sim.err || exit $?
done
