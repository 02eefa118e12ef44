#!/bin/bash
# r05: the stream / DTLS send frame kernels at one thread per record when the
# AEAD reads the content in place -- parity, then same-box A/B
set -o pipefail
O=gpurun_out/frame; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_stream_gpu.py tests/test_dtls_gpu.py tests/test_cid_gpu.py tests/test_evp_parity_gpu.py > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
bash tools/gpu_envab.sh frame TLSREC_LIBRARY=ablib/libtlsrec_gfni.so TLSREC_LIBRARY=ablib/libtlsrec_frame.so stream_cp dtls_cp stream16s dtls_small stream16
