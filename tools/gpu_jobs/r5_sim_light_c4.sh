# Round 5: C4 strong P = 8 (fused GIN passes) with light-row deferral off / 32 / 64, halo K 1 / 2,
# 400 GB/s, then the sharded GPU tests -> gpurun_out/r5slc
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5slc
mkdir -p $O
for L in 0 32 64; do
  KGX_HALO_LIGHT=$L timeout -k 10 300 python -u tools/shard_sim.py --config c4 --world 8 --steps 10 --chunks 1,2 --exchange halo --free-exchange --link-gbps 400 > $O/c4_l400_light$L.jsonl 2>> $O/err.log || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_sharded_fullsize.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
