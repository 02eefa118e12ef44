#!/bin/bash
# r05: E_K(J0) once per lane in the 16-wave key-pass kernels (all but G5) --
# parity, then same-box A/B
set -o pipefail
O=gpurun_out/ej0all; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_evp_parity_gpu.py tests/test_dtls_gpu.py tests/test_stream_gpu.py tests/test_gpu_parity.py tests/test_gpu_parity_edges.py tests/test_cid_gpu.py > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
bash tools/gpu_envab.sh ej0all TLSREC_LIBRARY=ablib/libtlsrec_ej0wp.so TLSREC_LIBRARY=ablib/libtlsrec_ej0all.so c4 c2s aria256 camellia128
