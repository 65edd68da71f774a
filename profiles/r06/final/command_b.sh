# Round 6 final measurement, part B: C3 / C4 / C5 kernel traces and PMC traffic
# (tools/gpu_jobs/gpu_pmc_configs.sh), the summaries copied into profiles/r06 on the box, then
# the C3 / C4 / C5 bench lines (traffic attached) and the strong-scaled NS form at N = 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O profiles/r06
bash tools/gpu_jobs/gpu_pmc_configs.sh c3 c4 c5 || exit $?
for c in c3 c4 c5; do
  cp gpurun_out/prof/pmc_$c.json profiles/r06/pmc_$c.json
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
done
timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/bench_ns_train.json 2> $O/bench_ns_train.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_train -o run \
  -- python3 bench.py --train --steps 10 --warmup 2 > $O/trace_train.log 2>&1 || exit $?
