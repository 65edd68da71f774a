# Round 3 (final sources): one rank's device work at weak P = 8 (NS), exchange-free and 400 GB/s links.
set -o pipefail
mkdir -p gpurun_out/r3sims
export TMPDIR=/tmp
: > gpurun_out/r3sims/ns_p8_final.jsonl
for L in 0 400; do
  timeout -k 10 500 python tools/shard_sim.py --config ns --world 8 --exchange halo --chunks 1,2 --merge-unit step,chunk \
    --link-gbps $L --steps 5 >> gpurun_out/r3sims/ns_p8_final.jsonl 2>> gpurun_out/r3sims/ns_final.err || exit $?
done
cat gpurun_out/r3sims/ns_p8_final.jsonl
