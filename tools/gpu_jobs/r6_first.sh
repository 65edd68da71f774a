# Round 6, first GPU session: the new GCN-norm parity tests (dinv table), the CU-split
# guard, the NS bench line on the changed sources, and one simulated NS weak P = 8 rank
# with the step's timeline (tools/shard_sim.py --timeline) plus the strong-scaled NS rows.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_gcn_norm.py tests/test_gpu_kernels.py tests/test_cu_split_host.py \
  "tests/test_gpu_layers.py::test_hip_graph_capture_cu_split" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_ns.json 2> $O/bench_ns.err || exit $?
S="python -u tools/shard_sim.py --config ns --world 8 --steps 10 --chunks 2 --exchange halo --free-exchange --timeline"
timeout -k 10 500 $S --link-gbps 400 --share-den 16,32 > $O/sim_ns_p8_400.jsonl 2> $O/sim.err || exit $?
timeout -k 10 500 $S --share-den 16 > $O/sim_ns_p8_free.jsonl 2>> $O/sim.err || exit $?
T="python -u tools/shard_sim.py --config ns_strong --steps 10 --exchange halo --free-exchange --link-gbps 400"
for P in 2 4 8; do
  timeout -k 10 400 $T --world $P --chunks 1,2 --share-den 16 > $O/sim_nsstrong_p$P.jsonl 2>> $O/sim.err || exit $?
done
