#!/bin/bash
# Lane / pass policy for 16 KiB records over many keys, same box: auto against
# forced wave passes at 4 and 16 lanes (TLSREC_GCM_LANES / TLSREC_GCM_WP).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/l16k
mkdir -p $O
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], d['metric'][:34], d['value'], d['check'])
" $1 $2; }
for i in 1 2; do
 for mode in auto wp4 wp16; do
  unset TLSREC_GCM_LANES TLSREC_GCM_WP
  [ $mode = wp4 ] && export TLSREC_GCM_LANES=4 TLSREC_GCM_WP=1
  [ $mode = wp16 ] && export TLSREC_GCM_LANES=16 TLSREC_GCM_WP=1
  for c in c4 k4; do
    timeout -k 10 300 python bench.py --config $c --no-cpu --no-e2e > $O/${c}_${mode}_$i.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['check'])" $O/${c}_${mode}_$i.json $c-$mode
  done
  timeout -k 10 200 python tools/bench_stream.py --conns 65536 --recs 16 > $O/s16_${mode}_$i.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
  show $O/s16_${mode}_$i.json stream16x16k-$mode
 done
done
