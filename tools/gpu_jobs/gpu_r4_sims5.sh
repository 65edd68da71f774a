#!/bin/bash
# Round 4: the new run-to-run bit-identity test, then NS weak P=8 one-rank
# simulations of pass A after the packs (KGX_HALO_A_LATE=2) against the layer's
# rule, repeated (sims job 4 gave 12.95 vs 14.86 ms at K 2 / step / 400 GB/s on
# one box, against 12.98 for the rule on another).
set -o pipefail
mkdir -p gpurun_out/r4s5
export TMPDIR=/tmp
O=gpurun_out/r4s5
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v -p no:cacheprovider --timeout 500 \
  --timeout-method thread -k "run_to_run" > $O/pytest_r2r.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_r2r.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 600 python tools/shard_sim.py --config ns --world 8 --chunks 2 --merge-unit step --a-late auto,2 \
    --steps 5 --link-gbps 400 --free-exchange >> $O/ns_400.jsonl 2>> $O/sim.err || exit $?
  timeout -k 10 600 python tools/shard_sim.py --config ns --world 8 --chunks 1 --merge-unit chunk,step --a-late 2,auto \
    --steps 5 --free-exchange >> $O/ns_free.jsonl 2>> $O/sim.err || exit $?
done
