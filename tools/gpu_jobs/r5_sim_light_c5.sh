# Round 5: C5 SAGE-mean strong P = 4 with light rows off / 32 (halo K 1 / 2, 400 GB/s), then the
# sharded GPU tests (threaded ranks on the HIP kernels) -> gpurun_out/r5sl5
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5sl5
mkdir -p $O
for L in 0 32; do
  KGX_HALO_LIGHT=$L timeout -k 10 300 python -u tools/shard_sim.py --config c5 --world 4 --steps 10 --chunks 1,2 --exchange halo --free-exchange --link-gbps 400 > $O/c5_l400_light$L.jsonl 2>> $O/err.log || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_sharded_fullsize.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
