# Round 5: NS CU split ratio (KGX_FUSED_FORK=3, KGX_FUSED_CU_SPLIT 4 / 8 / 12 / 16
# tail CUs per 32) against one stream, interleaved; kernel trace of the 8 split -> gpurun_out/nsc2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/nsc2
mkdir -p $O
for i in 1 2; do
  for c in 0 4 8 12 16; do
    if [ $c = 0 ]; then F=0; else F=3; fi
    KGX_FUSED_FORK=$F KGX_FUSED_CU_SPLIT=$c timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold \
      > $O/ns_split$c.$i.json 2> $O/ns_split$c.$i.err || exit $?
  done
done
KGX_FUSED_FORK=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/trace.log 2>&1 || exit $?
