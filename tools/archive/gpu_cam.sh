# Camellia-GCM/CCM GPU parity first, then the whole GPU suite, smoke, and benches
set -o pipefail
mkdir -p gpurun_out/cam
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "CAMELLIA or camellia" --timeout 120 --timeout-method thread > gpurun_out/cam/cam_tests.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cam/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/cam/smoke.txt 2>&1 || exit 1
for cfg in camellia128 c2 c4; do
timeout -k 10 300 python bench.py --no-cpu --config $cfg > gpurun_out/cam/bench_${cfg}.json 2>gpurun_out/cam/bench_${cfg}.err || exit 1
done
