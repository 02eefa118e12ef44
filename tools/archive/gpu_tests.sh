set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/gpu_tests.txt 2>&1
echo rc=$?
