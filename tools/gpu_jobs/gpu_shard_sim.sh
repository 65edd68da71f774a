# one-rank device-work simulation of the sharded GCN layer (tools/shard_sim.py) at several link rates
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/shard_sim.jsonl
for L in ${LINKS:-0 400}; do
  for pr in ${PRIOS:-1}; do
    KGX_SIDE_PRIORITY=$pr timeout -k 10 400 python tools/shard_sim.py --world ${WORLD:-8} --push 1 --chunks ${CHUNKS:-1,2,4} --link-gbps $L --steps 5 | sed "s/^{/{\"side_priority\": $pr, /" >> gpurun_out/shard_sim.jsonl || exit $?
  done
done
