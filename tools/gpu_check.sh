set -o pipefail
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m1 -E "gfx950" > gpurun_out/arch.txt || true
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config tiny --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_tiny.json 2> gpurun_out/bench_tiny.err
