#!/bin/bash
# Same-box A/B of two builds of libtlsrec.so over a few workloads.
#   tools/gpu_ab.sh <A.so> <B.so> -> gpurun_out/ab.txt
set -o pipefail
A=$1; B=$2; O=gpurun_out/ab.txt
: > $O
one() {  # lib tag cmd...
  local lib=$1 tag=$2; shift 2
  local v
  v=$(TLSREC_LIBRARY=$lib timeout -k 10 200 "$@" 2>/dev/null | python3 -c "
import sys,json
for l in sys.stdin:
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(d['metric'][:24].replace(' ','_'), d['value'])" | tr '\n' ' ') || return 1
  echo "$tag $(basename $lib) $v" >> $O
}
for round in 1 2; do
  for lib in $A $B; do
    one $lib c2 python3 bench.py --no-cpu --no-e2e --steps 10 || exit 1
    one $lib k4 python3 bench.py --config k4 --no-cpu --no-e2e --steps 5 || exit 1
    one $lib c4s python3 bench.py --config c4s --no-cpu --no-e2e --steps 5 || exit 1
    one $lib dtls1400 python3 tools/bench_dtls.py --steps 3 || exit 1
    one $lib streamcp python3 tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3 --steps 3 || exit 1
  done
done
cat $O
