# GPU suite, then same-box A/B (alternating order) of c2 / c3 / c4: tools_bin/libtlsrec_prev.so vs the current build
set -o pipefail
mkdir -p gpurun_out/ab3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || exit 1
for cfg in c3 c4 c2; do
timeout -k 10 300 python bench.py --no-cpu --config $cfg > gpurun_out/ab3/cur_${cfg}_1.json 2>/dev/null &&
TLSREC_LIBRARY=$PWD/tools_bin/libtlsrec_prev.so timeout -k 10 300 python bench.py --no-cpu --config $cfg > gpurun_out/ab3/prev_${cfg}_1.json 2>/dev/null &&
TLSREC_LIBRARY=$PWD/tools_bin/libtlsrec_prev.so timeout -k 10 300 python bench.py --no-cpu --config $cfg > gpurun_out/ab3/prev_${cfg}_2.json 2>/dev/null &&
timeout -k 10 300 python bench.py --no-cpu --config $cfg > gpurun_out/ab3/cur_${cfg}_2.json 2>/dev/null || exit 1
done
