# round 3: diagnose the degree-1 tiny kernel's bad rows on the NS graph (never-written rows,
# run-to-run differences, whether a bad row holds another row's result)
set -o pipefail
mkdir -p gpurun_out/r3t1c
export TMPDIR=/tmp
timeout -k 10 400 python tools/exp_tiny.py > gpurun_out/r3t1c/exp_tiny_main.log 2>&1; rc=$?; echo "main rc=$rc"
grep -v amdgpu.ids gpurun_out/r3t1c/exp_tiny_main.log | tail -8
