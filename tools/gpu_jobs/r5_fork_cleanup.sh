# Round 5: spmm.hip with the EXACT fork modes 1 / 2 removed (spmm_kernel ISA changed) against the
# previous library (lib/variants/libkgx_oldfork.so, built from the parent commit): C5 and NS EXACT bench
# lines interleaved, then the GPU suite + smoke + NS / C4 lines (tools/gpu_jobs/r5_suite2.sh) -> gpurun_out/fc
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/fc
mkdir -p $O
OLD=$PWD/keras-geometric_amd/lib/variants/libkgx_oldfork.so
for i in 1 2; do
  KGX_LIB=$OLD timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/c5_old.$i.json 2>> $O/err.log || exit $?
  timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/c5_new.$i.json 2>> $O/err.log || exit $?
  KGX_LIB=$OLD timeout -k 10 300 python bench.py --exact --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/exact_old.$i.json 2>> $O/err.log || exit $?
  timeout -k 10 300 python bench.py --exact --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/exact_new.$i.json 2>> $O/err.log || exit $?
done
bash tools/gpu_jobs/r5_suite2.sh
