#!/bin/bash
# Small-record GCM lane policy on one box: the -m gpu suite, the DTLS / stream
# 1.4 KiB AES-GCM rows under the auto policy, then forced 4-lane wave passes
# (TLSREC_GCM_LANES=4 TLSREC_GCM_WP=1) against auto on c4s and 64 records per key.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/l4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], d['metric'][:34], d['value'], d['check'])
" $1 $2; }
timeout -k 10 200 python tools/bench_dtls.py > $O/dtls_auto.json 2>$O/err.txt && show $O/dtls_auto.json dtls-auto &&
timeout -k 10 200 python tools/bench_stream.py --conns 65536 --recs 16 --content 1400 --cipher 2 > $O/stream_auto.json 2>$O/err.txt && show $O/stream_auto.json stream16x1.4k-auto || { tail -5 $O/err.txt; exit 1; }
for i in 1 2; do
 for mode in auto l4; do
  if [ $mode = l4 ]; then export TLSREC_GCM_LANES=4 TLSREC_GCM_WP=1; else unset TLSREC_GCM_LANES TLSREC_GCM_WP; fi
  timeout -k 10 300 python bench.py --config c4s --no-cpu --no-e2e > $O/c4s_${mode}_$i.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['check'])" $O/c4s_${mode}_$i.json c4s-$mode
  timeout -k 10 200 python tools/bench_stream.py --conns 16384 --recs 64 --content 1400 --cipher 2 > $O/s64_${mode}_$i.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
  show $O/s64_${mode}_$i.json stream64x1.4k-$mode
 done
done
unset TLSREC_GCM_LANES TLSREC_GCM_WP
