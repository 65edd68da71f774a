# Round 6: HBM traffic of one NS training step (FETCH_SIZE / WRITE_SIZE passes over the step's
# 12 launches, tools/pmc_step.py -> pmc_ns_train.json, copied into profiles/r06 on the box), then
# the training line with it attached.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6trpmc
mkdir -p $O profiles/r06
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run \
  --kernel-include-regex 'spmm_gemm|gemm_tn' -- python3 bench.py --train --steps 3 --warmup 1 > $O/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run \
  --kernel-include-regex 'spmm_gemm|gemm_tn' -- python3 bench.py --train --steps 3 --warmup 1 > $O/write.log 2>&1 || exit $?
F=$(find $O/fetch -name '*counter_collection.csv' | head -n 1)
W=$(find $O/write -name '*counter_collection.csv' | head -n 1)
python tools/pmc_step.py "$F" "$W" $O/pmc_ns_train.json --per-step 12 --steps 3 || exit $?
cp $O/pmc_ns_train.json profiles/r06/pmc_ns_train.json
timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 > $O/bench_train.json 2> $O/bench_train.err || exit $?
