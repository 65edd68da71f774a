# Round-5 profiles from the round-5 sources (one gpurun call): NS (bench line +
# rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes -> pmc_ns.json), the
# C3 / C4 / C5 configs (tools/gpu_jobs/gpu_pmc_configs.sh) and two SQ counter
# passes over the C4 fused 256-wide kernels (tools/exp_f256.py).  Outputs land in
# gpurun_out/prof; the summaries are then copied to profiles/r05/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/prof/bench_ns.json 2> gpurun_out/prof/bench_ns.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/prof/trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o run \
  --kernel-include-regex spmm -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/prof/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o run \
  --kernel-include-regex spmm -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/prof/write.log 2>&1 || exit $?
F=$(find gpurun_out/prof/fetch -name '*counter_collection.csv' | head -n 1)
W=$(find gpurun_out/prof/write -name '*counter_collection.csv' | head -n 1)
python tools/pmc_summary.py "$F" "$W" gpurun_out/prof/pmc_ns.json --config ns || exit $?
bash tools/gpu_jobs/gpu_pmc_configs.sh c3 c4 c5 || exit $?
# C4 fused 256-wide kernels: SQ counters (the tail's MFMA / VALU issue and waits)
PASS_A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"
PASS_B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD"
i=0
for P in "$PASS_A" "$PASS_B"; do
  i=$((i+1))
  KGX_EXP_UNFUSED=0 timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d gpurun_out/prof/f256sq$i -o run \
    --kernel-include-regex 'gemm256' -- python3 tools/exp_f256.py > gpurun_out/prof/f256sq$i.log 2>&1 || exit $?
done
