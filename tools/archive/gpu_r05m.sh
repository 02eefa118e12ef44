#!/bin/bash
# r05: stream / DTLS send reading the application data in place
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_stream_gpu.py tests/test_dtls_gpu.py tests/test_cid_gpu.py tests/test_evp_parity_gpu.py tests/test_gpu_parity.py tests/test_c_host.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
tools/gpu_envab.sh r05m/src TLSREC_STREAM_SRC=0 TLSREC_STREAM_SRC=1 stream16 stream16s stream4 dtls_small || exit 1
tools/gpu_ab_lib.sh r05m/lib ablib/libtlsrec_r05d.so mbedtls_amd/libtlsrec.so c3 c2se k4e c2 || exit 1
