#!/bin/bash
# r05: GCM kernel as two inlined lambdas (new lib) vs the lane-model build (ablib r05c), same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_evp_parity_gpu.py tests/test_stream_gpu.py tests/test_dtls_gpu.py tests/test_gpu_parity.py tests/test_gpu_parity_edges.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
tools/gpu_ab_lib.sh r05j/lib ablib/libtlsrec_r05c.so mbedtls_amd/libtlsrec.so c2 c2s c4 c4s k4 gcm192 c2 || exit 1
