#!/bin/bash
# r04: paired-pass lanes per record for 16 records per key (rule: 8) vs 4 and 2 -- DTLS and stream 1.4 KiB AES-GCM
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04pl}
mkdir -p $O
for rep in 1 2; do
  for l in 0 4 2; do
    if [ $l = 0 ]; then E="X=1"; else E="TLSREC_GCM_PAIR_L=$l"; fi
    env $E timeout -k 10 300 python3 tools/bench_dtls.py > $O/dtls_L${l}_$rep.json 2> $O/dtls_L${l}_$rep.err || { echo "dtls $l failed"; tail -3 $O/dtls_L${l}_$rep.err; exit 1; }
    env $E timeout -k 10 300 python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400 > $O/stream_L${l}_$rep.json 2> $O/stream_L${l}_$rep.err || { echo "stream $l failed"; exit 1; }
    echo L$l $(python3 -c "
import json,sys
for f in sys.argv[1:]:
    for l in open(f):
        l=l.strip()
        if l.startswith('{'): d=json.loads(l); print(d['metric'].split()[2] if 'DTLS' in d['metric'] else d['metric'].split()[1], d['value'], d['check'], end='; ')
" $O/dtls_L${l}_$rep.json $O/stream_L${l}_$rep.json)
  done
done
