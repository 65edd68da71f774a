#!/bin/bash
# Session re-entry check: smoke() on the rebuilt library, then the A_LATE=2 sims (gpu_r4_sims4.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4s1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4s1/smoke.log 2>&1 || exit $?
bash tools/gpu_jobs/gpu_r4_sims4.sh
