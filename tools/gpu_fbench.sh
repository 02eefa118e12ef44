# GPU tests, stream benches, c2/c3 regression (one box); outputs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 &&
timeout -k 10 300 python tools/bench_stream.py > gpurun_out/bench_stream.json 2> gpurun_out/bench_stream.err &&
timeout -k 10 300 python tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3 >> gpurun_out/bench_stream.json 2>> gpurun_out/bench_stream.err &&
timeout -k 10 300 python tools/bench_stream.py --conns 65536 --recs 4 --content 16384 --cipher 2 >> gpurun_out/bench_stream.json 2>> gpurun_out/bench_stream.err &&
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err &&
timeout -k 10 400 python bench.py --no-cpu --config c3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
echo rc=$?
