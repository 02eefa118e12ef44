# GPU parity + every bench config on one box; outputs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err &&
timeout -k 10 300 python bench.py --config c3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err &&
timeout -k 10 400 python bench.py --config c4 --no-cpu > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
echo rc=$?
