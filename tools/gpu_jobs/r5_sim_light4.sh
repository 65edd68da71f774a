# Round 5: NS weak P = 8 at 400 GB/s with light rows (default 32): K 1 / 2 / 4 x unit step / chunk,
# and compute alone at K 2 step -> gpurun_out/r5sl4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5sl4
mkdir -p $O
timeout -k 10 600 python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 1,2,4 --merge-unit step,chunk --exchange halo --free-exchange --link-gbps 400 > $O/l400.jsonl 2>> $O/err.log || exit $?
timeout -k 10 300 python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 2 --exchange halo --free-exchange > $O/free.jsonl 2>> $O/err.log || exit $?
