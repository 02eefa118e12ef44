#!/bin/bash
# Table-free lane tree for 16-lane wave passes (TLSREC_GCM_TREEMUL=1) against
# the HBM tree tables, same box: parity of the wave-pass tests with it on,
# then k4 / k4e / stream 4 x 16 KiB per key with 0 / 1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/tm
mkdir -p $O
TLSREC_GCM_TREEMUL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_edges.py tests/test_stream_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], d['metric'][:34], d['value'], d['check'])
" $1 $2; }
for i in 1 2; do
 for v in 0 1; do
  export TLSREC_GCM_TREEMUL=$v
  for c in k4 k4e; do
    timeout -k 10 300 python bench.py --config $c --no-cpu --no-e2e > $O/${c}_${v}_$i.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['check'])" $O/${c}_${v}_$i.json $c-tm$v
  done
  timeout -k 10 200 python tools/bench_stream.py --conns 65536 --recs 4 > $O/s4_${v}_$i.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
  show $O/s4_${v}_$i.json stream4x16k-tm$v
 done
done
