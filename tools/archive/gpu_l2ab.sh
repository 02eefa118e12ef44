#!/bin/bash
# 2-lane against 4-lane (auto) wave passes for small records, same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/l2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wave_pass" > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], d['metric'][:34], d['value'], d['check'])
" $1 $2; }
for i in 1 2; do
 for mode in auto l2; do
  unset TLSREC_GCM_LANES TLSREC_GCM_WP
  [ $mode = l2 ] && export TLSREC_GCM_LANES=2 TLSREC_GCM_WP=1
  timeout -k 10 300 python bench.py --config c4s --no-cpu --no-e2e > $O/c4s_${mode}_$i.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['check'])" $O/c4s_${mode}_$i.json c4s-$mode
  timeout -k 10 200 python tools/bench_stream.py --conns 16384 --recs 64 --content 1400 --cipher 2 > $O/s64_${mode}_$i.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
  show $O/s64_${mode}_$i.json stream64x1.4k-$mode
  timeout -k 10 200 python tools/bench_dtls.py > $O/dtls_${mode}_$i.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
  show $O/dtls_${mode}_$i.json dtls16x1.4k-$mode
 done
done
