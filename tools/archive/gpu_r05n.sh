#!/bin/bash
# r05: ChaCha src mode as a template flag; c3 regression check and send rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_stream_gpu.py tests/test_dtls_gpu.py tests/test_cid_gpu.py tests/test_gpu_parity.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
tools/gpu_ab_lib.sh r05n/lib ablib/libtlsrec_r05d.so mbedtls_amd/libtlsrec.so c3 c3 chacha16ke c2se || exit 1
tools/gpu_envab.sh r05n/src TLSREC_STREAM_SRC=0 TLSREC_STREAM_SRC=1 stream_cp dtls_cp || exit 1
