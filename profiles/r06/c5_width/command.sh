# Round 6: C5's 1.08x fetched bytes -- the 64-byte sector claim tested by
# row WIDTH: kgx_spmm_ex2 MEAN over the C5 graph with F = 96 / 100 / 112 / 128 (ld = F),
# time and FETCH_SIZE per launch (own rocprofv3 pass each).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6c5
mkdir -p $O
for F in 96 100 112 128; do
  timeout -k 10 300 python tools/exp_c5_stride.py --features $F >> $O/c5_width.jsonl 2>> $O/c5.err || exit $?
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$F -o run \
    --kernel-include-regex spmm -- python3 tools/exp_c5_stride.py --features $F --reps 3 > $O/pmc_$F.log 2>&1 || exit $?
done
