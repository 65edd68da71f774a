# Round 5: CU-split mask pattern A/B (first 8 of every 32 CUs vs 2 of every 8), NS and C4,
# three interleaved rounds -> gpurun_out/cpat
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/cpat
mkdir -p $O
for i in 1 2 3; do
  for p in 0 1; do
    KGX_CU_SPLIT_INTERLEAVE=$p timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > $O/ns_p$p.$i.json 2>> $O/err.log || exit $?
    KGX_CU_SPLIT_INTERLEAVE=$p timeout -k 10 200 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/c4_p$p.$i.json 2>> $O/err.log || exit $?
  done
done
