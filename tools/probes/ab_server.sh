#!/bin/bash
# same-box A/B of the record server's AES form: rolled (default) vs unrolled
set -o pipefail
mkdir -p gpurun_out/ab
: > gpurun_out/ab/out.txt
for v in rolled unrolled rolled unrolled; do
  for a in "latency 2 1.3 1400 1000" "latency 2 1.3 16383 500" "threads 16 2000 gcm_chacha"; do
    echo "$v $a $(TLSREC_SERVER_AES=$v timeout -k 5 60 ./tests/c/abi_host $a)" >> gpurun_out/ab/out.txt || exit 1
  done
done
cat gpurun_out/ab/out.txt
