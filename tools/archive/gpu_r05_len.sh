#!/bin/bash
# r05: the LEN Horner step by the pass's LDS table -- parity, then same-box A/B
set -o pipefail
mkdir -p gpurun_out/len
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_evp_parity_gpu.py tests/test_dtls_gpu.py tests/test_stream_gpu.py tests/test_gpu_parity.py > gpurun_out/len/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/len/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/len/gpu_tests.txt
bash tools/gpu_ab_lib.sh len ablib/libtlsrec_prelen.so ablib/libtlsrec_len.so k4 c2s
