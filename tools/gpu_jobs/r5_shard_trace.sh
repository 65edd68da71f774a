# Round 5: kernel trace of one rank of NS weak P = 8 (halo K 2, unit step, 400 GB/s modelled link)
# and C4 strong P = 8 (halo K 2, step) -> gpurun_out/strace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/strace
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ns -o run -- python3 tools/shard_sim.py --config ns --world 8 --steps 5 --chunks 2 --exchange halo --free-exchange --link-gbps 400 > $O/ns.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 tools/shard_sim.py --config c4 --world 8 --steps 5 --chunks 2 --exchange halo --free-exchange --link-gbps 400 > $O/c4.log 2>&1 || exit $?
