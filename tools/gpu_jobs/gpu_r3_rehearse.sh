# round 3: bench.py's N>1 path rehearsed on one GPU (2 ranks, host-staged gloo exchange): GCN weak (c2)
# with the exchange autotuner at the first forward; GIN C4 and SAGE C5 strong at fixed K (the host-staged
# exchange of GBs per tuning forward would take minutes); control flow only, never a measurement
set -o pipefail
mkdir -p gpurun_out/r3reh
export TMPDIR=/tmp
KGX_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --config c2 --steps 2 --warmup 1 \
  > gpurun_out/r3reh/c2.json 2> gpurun_out/r3reh/c2.err || { tail -30 gpurun_out/r3reh/c2.err; exit 1; }
for c in c4 c5; do
  KGX_HALO_CHUNKS=2 KGX_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --config $c --steps 2 --warmup 1 \
    > gpurun_out/r3reh/$c.json 2> gpurun_out/r3reh/$c.err || { tail -30 gpurun_out/r3reh/$c.err; exit 1; }
done
KGX_EXCHANGE=allgather KGX_HALO_CHUNKS=2 KGX_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --config c5 \
  --steps 2 --warmup 1 > gpurun_out/r3reh/c5_allgather.json 2> gpurun_out/r3reh/c5_allgather.err || { tail -30 gpurun_out/r3reh/c5_allgather.err; exit 1; }
