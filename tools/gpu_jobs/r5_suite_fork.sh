# Round 5: GPU suite (-> gpurun_out/r5a) then the NS fork A/B (tools/gpu_jobs/r5_ab_fork.sh
# body: KGX_FUSED_FORK 0 / 1 / 2, three interleaved bench lines each -> gpurun_out/r5b).
# A failing test does not stop the A/B; a fault, abort or time-out does.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5a gpurun_out/r5b
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5a/pytest.log 2>&1
rc=$?
echo "pytest rc $rc" >> gpurun_out/r5a/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  for f in 0 1 2; do
    KGX_FUSED_FORK=$f timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold \
      > gpurun_out/r5b/ns_fork$f.$i.json 2> gpurun_out/r5b/ns_fork$f.$i.err || exit $?
  done
done
exit $rc
