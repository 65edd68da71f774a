# round-3 first probe: GATv2 backward seed sweep + a kernel trace of the weak P=8 shard simulation
set -o pipefail
mkdir -p gpurun_out/r3probe
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/exp_gatv2_seeds.py ${SEEDS:-48} > gpurun_out/r3probe/gatv2_seeds.jsonl 2> gpurun_out/r3probe/gatv2_seeds.err || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3probe/sim -o run \
  -- python3 tools/shard_sim.py --world 8 --push 1 --chunks 1 --steps 3 > gpurun_out/r3probe/sim.jsonl 2> gpurun_out/r3probe/sim.err || exit $?
