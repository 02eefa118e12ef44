# same-box A/B of ChaCha20-Poly1305 kernel variants on c3 (libs in tools_bin/)
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "CHACHA or many_keys or mixed or large" > gpurun_out/ab/tests.txt 2>&1 || exit 1
for i in 1 2; do
  for v in prev b c d; do
    TLSREC_LIBRARY=$PWD/tools_bin/libtlsrec_$v.so timeout -k 10 300 python bench.py --no-cpu --config c3 > gpurun_out/ab/c3_${v}_$i.json 2>/dev/null || exit 1
  done
done
echo rc=$?
