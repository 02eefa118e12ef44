#!/bin/bash
# record-server debugging: consecutive C processes with a request trace
set -o pipefail
mkdir -p gpurun_out/dbg
for a in "2 1.3 16383 50" "2 1.3 1400 50" "3 1.3 1400 50"; do
  echo "== $a" >> gpurun_out/dbg/seq.txt
  TLSREC_SERVER_DEBUG=1 AMD_LOG_LEVEL=1 timeout -k 5 60 ./tests/c/abi_host latency $a > gpurun_out/dbg/out.txt 2> gpurun_out/dbg/err.txt
  rc=$?
  echo "rc=$rc" >> gpurun_out/dbg/seq.txt
  cat gpurun_out/dbg/out.txt >> gpurun_out/dbg/seq.txt
  grep -v "slot 0 seq" gpurun_out/dbg/err.txt | tail -20 >> gpurun_out/dbg/seq.txt
  head -3 gpurun_out/dbg/err.txt >> gpurun_out/dbg/seq.txt
  [ $rc -ne 0 ] && break
done
cat gpurun_out/dbg/seq.txt
