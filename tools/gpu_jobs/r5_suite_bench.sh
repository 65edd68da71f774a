set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5a
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5a/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r5a/bench_ns.json 2> gpurun_out/r5a/bench_ns.err
