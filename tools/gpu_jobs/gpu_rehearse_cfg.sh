# N>1 control-flow rehearsal of the C4 / C5 strong-scaled sharded layers through
# bench.py's own launcher (2 ranks sharing the one GPU, exchange staged over gloo):
# exercises ShardedGINConv / ShardedSAGEConv end to end on hardware; never a measurement.
set -o pipefail
mkdir -p gpurun_out/reh
for c in c4 c5; do
  KGX_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --config $c --steps 2 --warmup 1 > gpurun_out/reh/$c.json 2> gpurun_out/reh/$c.err || { tail -20 gpurun_out/reh/$c.err; exit 1; }
done
cat gpurun_out/reh/*.json
