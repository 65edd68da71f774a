# round 3: merged-halo sharded layers -- GPU distributed + full-size sharded tests, NS bench, P=8 simulation
set -o pipefail
mkdir -p gpurun_out/r3shard
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_distributed.py \
  tests/test_gpu_sharded_fullsize.py tests/test_gpu_dense.py tests/test_gpu_tiny.py tests/test_gpu_layers.py -s > gpurun_out/r3shard/pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/r3shard/bench_ns.json 2> gpurun_out/r3shard/bench_ns.err || exit $?
: > gpurun_out/r3shard/sim.jsonl
for L in ${LINKS:-0 400}; do
  timeout -k 10 400 python tools/shard_sim.py --config ns --world 8 --merged ${MERGED:-1,0} --chunks ${CHUNKS:-1,2} \
    --link-gbps $L --steps 5 >> gpurun_out/r3shard/sim.jsonl 2>> gpurun_out/r3shard/sim.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3shard/trace -o run \
  -- python3 tools/shard_sim.py --world 8 --merged 1 --chunks 1 --steps 3 > gpurun_out/r3shard/trace.log 2>&1 || exit $?
KGX_AB_WORK=gat timeout -k 10 600 python tools/exp_agg.py ab main main:KGX_GAT_K=8 main:KGX_GAT_K=16 gu2:KGX_GAT_K=16 gu4:KGX_GAT_K=16 gu4 > gpurun_out/r3shard/gat_ab.log 2>&1 || exit $?
