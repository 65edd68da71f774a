# round 3 batch: parity (GATv2 K=8, EXACT fork/join, distributed), NS/EXACT bench, fused A/B, shard sims
set -o pipefail
mkdir -p gpurun_out/r3b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_layers.py tests/test_gpu_backward.py tests/test_gatv2_conditioning.py tests/test_gpu_distributed.py \
  tests/test_gpu_configs.py > gpurun_out/r3b/pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/r3b/bench_ns.json 2> gpurun_out/r3b/bench_ns.err || exit $?
timeout -k 10 300 python bench.py --exact --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/r3b/bench_exact.json 2> gpurun_out/r3b/bench_exact.err || exit $?
KGX_AB_WORK=both timeout -k 10 600 python tools/exp_agg.py ab main oldchk > gpurun_out/r3b/ab_fused.log 2>&1 || exit $?
: > gpurun_out/r3b/sim_ns.jsonl
for L in 0 400; do
  timeout -k 10 600 python tools/shard_sim.py --config ns --world 8 --merged 1 --merge-unit step,chunk --a-late 0,1 \
    --chunks 1,2,4 --link-gbps $L --steps 5 >> gpurun_out/r3b/sim_ns.jsonl 2>> gpurun_out/r3b/sim.err || exit $?
done
