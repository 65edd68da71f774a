# Round 3 (final sources): repeat of the best exchange-free NS weak P = 8 configuration (K 1, unit chunk) for its spread.
set -o pipefail
mkdir -p gpurun_out/r3sims
export TMPDIR=/tmp
: > gpurun_out/r3sims/ns_p8_k1_repeat.jsonl
timeout -k 10 500 python tools/shard_sim.py --config ns --world 8 --exchange halo --chunks 1 --merge-unit chunk \
  --link-gbps 0 --steps 10 >> gpurun_out/r3sims/ns_p8_k1_repeat.jsonl 2>> gpurun_out/r3sims/ns_k1.err || exit $?
cat gpurun_out/r3sims/ns_p8_k1_repeat.jsonl
