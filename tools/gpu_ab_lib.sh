#!/bin/bash
# Same-box A/B of two in-tree builds of libtlsrec:
#   tools/gpu_ab_lib.sh <outdir> <libA.so> <libB.so> <config>...
# Each config runs A, B, B, A (bench.py --no-cpu --no-e2e, 10 timed steps);
# prints value and kernel ms per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/$1; A=$2; B=$3; shift 3
mkdir -p $O
for c in "$@"; do
  for lib in $A $B $B $A; do
    tag=$(basename $lib .so)
    TLSREC_LIBRARY=$R/$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-e2e --verify 16 > $O/$c.$tag.json 2> $O/$c.$tag.err || { echo "FAIL $c $tag"; tail -3 $O/$c.$tag.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['roofline']['kernel_ms_avg'], d['check']['bad_records'])" $O/$c.$tag.json $c $tag
  done
done
