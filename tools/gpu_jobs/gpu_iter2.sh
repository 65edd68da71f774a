# quick iteration: full GPU suite + rocprof kernel stats of the given configs (default c3 c5 ns)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/it
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/it/tests.log 2>&1 || exit $?
for c in ${CONFIGS:-c3 c5 ns}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/it/trace_$c -o run \
    -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/it/bench_$c.json 2> gpurun_out/it/bench_$c.err || exit $?
done
