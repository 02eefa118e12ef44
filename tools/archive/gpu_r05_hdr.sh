#!/bin/bash
# r05: stream receive header walk with one 8-byte load per header -- parity, then A/B
set -o pipefail
O=gpurun_out/hdr; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_stream_gpu.py tests/test_ticket_gpu.py > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
bash tools/gpu_envab.sh hdr TLSREC_LIBRARY=ablib/libtlsrec_fin.so TLSREC_LIBRARY=ablib/libtlsrec_hdr.so stream_cp stream16s
