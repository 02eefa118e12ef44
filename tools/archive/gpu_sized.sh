#!/bin/bash
# Size-hinted small-record policy on one box: the -m gpu suite, then the rows
# it changes (c4s, 64 and 16 records per key through the stream / DTLS layers)
# and the BASELINE configs it must not change.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/sz
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], d['metric'][:34], d['value'], d['check'])
" $1 $2; }
for c in c4s c4 k4 c2 c3; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-e2e > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['frac'], d['check'])" $O/$c.json $c
done
timeout -k 10 200 python tools/bench_stream.py --conns 16384 --recs 64 --content 1400 --cipher 2 > $O/s64.json 2>$O/err.txt && show $O/s64.json stream64x1.4k &&
timeout -k 10 200 python tools/bench_stream.py --conns 65536 --recs 16 --content 1400 --cipher 2 > $O/s16.json 2>$O/err.txt && show $O/s16.json stream16x1.4k &&
timeout -k 10 200 python tools/bench_dtls.py > $O/dtls.json 2>$O/err.txt && show $O/dtls.json dtls16x1.4k || { tail -5 $O/err.txt; exit 1; }
