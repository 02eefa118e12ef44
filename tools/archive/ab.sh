# same-box A/B: tools_bin/libtlsrec_prev.so (an earlier build of the ABI) vs the current build
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.txt 2>&1 || exit 1
for i in 1 2; do
TLSREC_LIBRARY=$PWD/tools_bin/libtlsrec_prev.so timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/ab/prev_$i.json 2>/dev/null &&
timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/ab/cur_$i.json 2>/dev/null || exit 1
done
