# Round 5: GPU suite + NS bench line (-> gpurun_out/r5a), then the C4 tail
# (spmm_gemm256_tiny2_kernel) wave-order A/B: shipped / waves 4-7 MFMA-first
# (KGX_T2_STAGGER) / waves 4-7 at s_setprio 1 (KGX_T2_PRIO) / both; three
# interleaved rounds of tools/exp_f256.py (-> gpurun_out/t2ab).  A failing test
# does not stop the A/B; a fault, abort or time-out does.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5a gpurun_out/t2ab
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5a/pytest.log 2>&1
rc=$?
echo "pytest rc $rc" >> gpurun_out/r5a/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/r5a/bench_ns.json 2> gpurun_out/r5a/bench_ns.err || exit $?
: > gpurun_out/t2ab/ab.log
for round in 0 1 2; do
  for lib in main t2stag t2prio t2both; do
    if [ $lib = main ]; then L=keras-geometric_amd/lib/libkgx.so; else L=keras-geometric_amd/lib/variants/libkgx_$lib.so; fi
    KGX_EXP_UNFUSED=0 KGX_LIB=$L timeout -k 10 240 python tools/exp_f256.py >> gpurun_out/t2ab/ab.log 2> gpurun_out/t2ab/$lib.err || exit $?
  done
done
exit $rc
