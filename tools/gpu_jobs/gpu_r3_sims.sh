# round 3: one-rank device-work simulations of the strong-scaled configs (C4 GIN-sum P=8, C5 SAGE-mean P=4),
# push-pull halo vs all-gather, exchange-free and with modelled links
set -o pipefail
mkdir -p gpurun_out/r3sims
export TMPDIR=/tmp
: > gpurun_out/r3sims/c4_p8.jsonl
: > gpurun_out/r3sims/c5_p4.jsonl
for L in 0 400; do
  timeout -k 10 400 python tools/shard_sim.py --config c4 --world 8 --exchange halo,allgather --chunks 1,2 \
    --link-gbps $L --steps 5 >> gpurun_out/r3sims/c4_p8.jsonl 2>> gpurun_out/r3sims/sim.err || exit $?
done
for L in 0 170 400; do
  timeout -k 10 400 python tools/shard_sim.py --config c5 --world 4 --exchange halo,allgather --chunks 1,2,4 \
    --link-gbps $L --steps 5 >> gpurun_out/r3sims/c5_p4.jsonl 2>> gpurun_out/r3sims/sim.err || exit $?
done
