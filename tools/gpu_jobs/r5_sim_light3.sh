# Round 5: light-row bound sweep (KGX_HALO_LIGHT 0 / 7 / 12 / 20, two rounds), NS weak P = 8, halo K 2,
# 400 GB/s; and C4 strong P = 8 halo K 2 (the GIN path does not defer: unchanged) -> gpurun_out/r5sl3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5sl3
mkdir -p $O
for round in 1 2; do
  for L in 20 32 48 64; do
    KGX_HALO_LIGHT=$L timeout -k 10 300 python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 2 --exchange halo --free-exchange --link-gbps 400 > $O/l400_light$L.$round.jsonl 2>> $O/err.log || exit $?
  done
done
