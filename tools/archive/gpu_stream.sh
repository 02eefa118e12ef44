set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_stream_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/stream_tests.txt 2>&1
echo rc=$?
