#!/bin/bash
# same-box A/B of two builds of libtlsrec.so over bench rows:
#   tools/probes/ab_lib.sh <other.so> <config>...   (runs new, old, old, new)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
OLD=$1; shift
for cfg in "$@"; do
for lib in new old old new; do
  if [ $lib = old ]; then L=$OLD; else L=mbedtls_amd/libtlsrec.so; fi
  TLSREC_LIBRARY=$L timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-e2e --verify 16 > gpurun_out/ab.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$cfg', '$lib', d['value'], d['check']['bad_records'])"
done; done
