#!/bin/bash
# r05: E_K(J0) once per lane in the paired kernels -- parity, then same-box A/B
set -o pipefail
mkdir -p gpurun_out/ej0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_evp_parity_gpu.py tests/test_dtls_gpu.py tests/test_stream_gpu.py tests/test_gpu_parity.py > gpurun_out/ej0/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/ej0/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/ej0/gpu_tests.txt
bash tools/gpu_envab.sh ej0 TLSREC_LIBRARY=ablib/libtlsrec_len.so TLSREC_LIBRARY=ablib/libtlsrec_ej0.so dtls_small stream16s k4 c4s stream16
