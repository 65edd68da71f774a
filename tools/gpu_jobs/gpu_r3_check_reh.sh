# round 3: full GPU suite, then bench.py's N>1 path rehearsed on the one GPU (tools/gpu_jobs/gpu_r3_rehearse.sh)
set -o pipefail
mkdir -p gpurun_out/r3chk
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3chk/pytest.log 2>&1 || { tail -40 gpurun_out/r3chk/pytest.log; exit 1; }
tail -3 gpurun_out/r3chk/pytest.log
bash tools/gpu_jobs/gpu_r3_rehearse.sh || exit $?
for f in gpurun_out/r3reh/*.json; do echo "$f: $(cut -c1-300 $f)"; done
