# Bench lines (PMC traffic attached from the newest profiles/r*) for NS and the C3/C4/C5 configs.
set -o pipefail
mkdir -p gpurun_out/lines
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/lines/bench_ns.json 2> gpurun_out/lines/bench_ns.err || exit $?
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cold > gpurun_out/lines/bench_$c.json 2> gpurun_out/lines/bench_$c.err || exit $?
done
