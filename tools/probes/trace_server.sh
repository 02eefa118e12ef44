#!/bin/bash
# record-server parity tests, then phase times (device wall clock) and latency for lone records
set -o pipefail
mkdir -p gpurun_out/trace
timeout -k 10 300 python -u -m pytest tests/test_server_gpu.py tests/test_fail_closed_gpu.py tests/test_coalesce_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/trace/tests.txt 2>&1 || { tail -30 gpurun_out/trace/tests.txt; exit 1; }
tail -1 gpurun_out/trace/tests.txt
: > gpurun_out/trace/out.txt
for a in "2 1.3 1400" "3 1.3 1400" "2 1.3 100" "2 1.3 16383" "3 1.3 16383"; do
  TLSREC_SERVER_TRACE=1 timeout -k 5 60 ./tests/c/abi_host latency $a 1000 >> gpurun_out/trace/out.txt 2>&1 || exit 1
done
for t in 16 32; do timeout -k 5 60 ./tests/c/abi_host threads $t 2000 gcm_chacha >> gpurun_out/trace/out.txt 2>&1 || exit 1; done
cat gpurun_out/trace/out.txt
