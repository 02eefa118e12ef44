#!/bin/bash
# A/B two libtlsrec.so builds on the ChaCha20-Poly1305 rows -> gpurun_out/ab_cp.txt
set -o pipefail
A=$1; B=$2; O=gpurun_out/ab_cp.txt
: > $O
for round in 1 2; do
  for lib in $A $B; do
    for cfg in c3 chacha16k; do
      v=$(TLSREC_LIBRARY=$lib timeout -k 10 200 python3 bench.py --config $cfg --no-cpu --no-e2e --steps 10 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms_avg'], d['check']['bad_records'])") || exit 1
      echo "$cfg $(basename $lib) $v" >> $O
    done
  done
done
cat $O
