#!/bin/bash
# r05: the table-free GF(2^128) multiply with three-input XORs, masked merges
# and builtin bit reversal -- parity (every file whose kernels multiply
# table-free: GCM lane powers, wave-pass trees, the record server), then A/B
set -o pipefail
O=gpurun_out/gf; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_evp_parity_gpu.py tests/test_dtls_gpu.py tests/test_stream_gpu.py tests/test_gpu_parity.py tests/test_gpu_parity_edges.py tests/test_cid_gpu.py tests/test_server_gpu.py > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
bash tools/gpu_envab.sh gf TLSREC_LIBRARY=ablib/libtlsrec_pregf.so TLSREC_LIBRARY=ablib/libtlsrec_gf.so dtls_small stream16s c4s k4
