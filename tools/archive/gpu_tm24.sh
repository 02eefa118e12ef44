#!/bin/bash
# Table-free lane tree in the 2- and 4-lane wave passes (TLSREC_GCM_TREEMUL=3)
# against the HBM tree tables (=1, default), same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/tm24
mkdir -p $O
TLSREC_GCM_TREEMUL=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wave_pass or sized" > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], d['metric'][:34], d['value'], d['check'])
" $1 $2; }
for i in 1 2; do
 for v in 1 3; do
  export TLSREC_GCM_TREEMUL=$v
  timeout -k 10 200 python tools/bench_dtls.py > $O/d_${v}_$i.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
  show $O/d_${v}_$i.json dtls16x1.4k-tm$v
  timeout -k 10 300 python bench.py --config c4s --no-cpu --no-e2e > $O/c4s_${v}_$i.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['check'])" $O/c4s_${v}_$i.json c4s-tm$v
 done
done
