set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.txt 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.txt 2>&1 &&
timeout -k 10 300 python tools/e2e.py > gpurun_out/e2e.txt 2>&1
echo rc=$?
