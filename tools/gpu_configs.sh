set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || exit $?
