#!/bin/bash
# GCM launch policy: default vs wave passes at L=16, over records per key and record size
set -e
O=gpurun_out/rpk.txt
: > $O
for args in "--config k4 --records 1048576" "--config k4 --records 2097152" "--config k4" "--config c4s" "--config c4s --records 1048576" "--config c4"; do
  for v in "" "TLSREC_GCM_WP=1 TLSREC_GCM_LANES=16"; do
    r=$(env $v timeout -k 10 120 python -u bench.py $args --steps 3 --warmup 1 --no-cpu --no-e2e --verify 8 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['records_per_gpu'], d['check']['bad_records'])")
    echo "$args | $v | $r" >> $O
  done
done
