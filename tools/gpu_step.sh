set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools_bin/prim_probe > gpurun_out/probe.txt 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.txt 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.txt 2>&1 &&
TLSREC_GCM_WAVES=8 timeout -k 10 300 python bench.py > gpurun_out/bench_w8.txt 2>&1
echo rc=$?
