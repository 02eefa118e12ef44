#!/bin/bash
# r05: no bucket pass for ChaCha20-Poly1305-only key tables -- parity, then A/B
set -o pipefail
O=gpurun_out/nobucket; mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_stream_gpu.py tests/test_dtls_gpu.py tests/test_fail_closed_gpu.py tests/test_gpu_parity.py tests/test_evp_parity_gpu.py tests/test_gpu_parity_edges.py tests/test_engine_hygiene_gpu.py tests/test_cid_gpu.py > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
bash tools/gpu_envab.sh nobucket TLSREC_LIBRARY=ablib/libtlsrec_frame.so TLSREC_LIBRARY=ablib/libtlsrec_nobucket.so stream_cp dtls_cp c4s
