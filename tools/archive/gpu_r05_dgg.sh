#!/bin/bash
# r05: the DTLS test file on the in-tree build; then the variant with the
# receive count / emit walks at 16 lanes per connection (ablib/libtlsrec_dgg.so):
# its parity, and a same-box A/B against the in-tree build
set -o pipefail
O=gpurun_out/dgg; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_dtls_gpu.py > $O/gpu_tests_final.txt 2>&1 || { tail -30 $O/gpu_tests_final.txt; exit 1; }
tail -1 $O/gpu_tests_final.txt
TLSREC_LIBRARY=ablib/libtlsrec_dgg.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_dtls_gpu.py tests/test_cid_gpu.py > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
bash tools/gpu_envab.sh dgg TLSREC_LIBRARY=ablib/libtlsrec_fin.so TLSREC_LIBRARY=ablib/libtlsrec_dgg.so dtls_cp dtls_small
