# full GPU suite, then same-box A/B of c2 / c3: tools_bin/libtlsrec_prev.so vs the current build
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || exit 1
for cfg in c2 c3; do
for i in 1 2; do
TLSREC_LIBRARY=$PWD/tools_bin/libtlsrec_prev.so timeout -k 10 300 python bench.py --no-cpu --config $cfg > gpurun_out/ab/prev_${cfg}_$i.json 2>/dev/null &&
timeout -k 10 300 python bench.py --no-cpu --config $cfg > gpurun_out/ab/cur_${cfg}_$i.json 2>/dev/null || exit 1
done
done
