set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_keysched_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/ks_tests.txt 2>&1 &&
timeout -k 10 300 python bench.py --config c1 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err
echo rc=$?
