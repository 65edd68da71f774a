# Round 5: with light rows (default 32), the own-only pass order (KGX_HALO_A_LATE auto / 0 / 1) at
# NS weak P = 8, 400 GB/s, halo K 2 step and K 4 chunk, two rounds -> gpurun_out/r5sa
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5sa
mkdir -p $O
S="python -u tools/shard_sim.py --config ns --world 8 --steps 10 --exchange halo --free-exchange --link-gbps 400"
for round in 1 2; do
  for A in auto 0 1; do
    timeout -k 10 300 $S --chunks 2 --merge-unit step --a-late $A > $O/k2step_alate$A.$round.jsonl 2>> $O/err.log || exit $?
    timeout -k 10 300 $S --chunks 4 --merge-unit chunk --a-late $A > $O/k4chunk_alate$A.$round.jsonl 2>> $O/err.log || exit $?
  done
done
