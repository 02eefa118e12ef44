#!/bin/bash
# r05: paired 16-lane passes vs 16-wave key passes for 16 KiB records, 12..64 per key
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05e; mkdir -p $O
for k in 21846 16384 10923 8192 5462 4096; do
  for v in 0 16 16 0; do
    TLSREC_GCM_PAIR_BIG=$v timeout -k 10 300 python3 bench.py --config k4 --keys $k --records 262144 --no-cpu --no-e2e --verify 16 > $O/k$k.$v.json 2> $O/k$k.$v.err || { tail -3 $O/k$k.$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'rpk', 262144 // int(sys.argv[2]), 'pair_big', sys.argv[3], d['value'], d['check']['bad_records'])" $O/k$k.$v.json $k $v
  done
done
