#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05l; mkdir -p $O
for v in 1 0 0 1; do
  TLSREC_HOST_ZC=$v timeout -k 10 300 python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/e2e.$v.json 2> $O/e2e.$v.err || { tail -5 $O/e2e.$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('zc', sys.argv[2], d['e2e'])" $O/e2e.$v.json $v
done
