# Round 5: NS weak P = 8, halo K 2 / 4 (unit step), light-row deferral KGX_HALO_LIGHT
# 0 / 2 / 7 / 10^5; compute alone and 400 GB/s -> gpurun_out/r5sl
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5sl
mkdir -p $O
for L in 0 7 2 100000; do
  KGX_HALO_LIGHT=$L timeout -k 10 300 python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 2,4 --exchange halo --free-exchange --link-gbps 400 > $O/l400_light$L.jsonl 2>> $O/err.log || exit $?
done
for L in 0 7; do
  KGX_HALO_LIGHT=$L timeout -k 10 300 python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 2 --exchange halo --free-exchange > $O/free_light$L.jsonl 2>> $O/err.log || exit $?
done
