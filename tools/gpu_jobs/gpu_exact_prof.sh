set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ex
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ex/trace -o run -- python3 bench.py --exact --steps 5 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/ex/bench.json 2> gpurun_out/ex/bench.err
