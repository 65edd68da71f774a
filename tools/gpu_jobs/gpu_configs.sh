# Per-config timings (tools/bench_configs.py) for one GPU call; output -> gpurun_out/configs.jsonl
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/bench_configs.py "$@" > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
