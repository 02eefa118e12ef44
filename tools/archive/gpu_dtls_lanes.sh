#!/bin/bash
# DTLS small-datagram AES-GCM receive: lanes-per-record / wave-pass variants
set -e
for v in "" "TLSREC_GCM_WP=1" "TLSREC_GCM_LANES=16" "TLSREC_GCM_LANES=16 TLSREC_GCM_WP=1" "TLSREC_GCM_LANES=8"; do
  echo "== $v" >> gpurun_out/dtls_lanes.txt
  env $v timeout -k 10 120 python -u tools/bench_dtls.py --steps 3 >> gpurun_out/dtls_lanes.txt 2>&1
done
