#!/bin/bash
# r05: small records (1 400 B AES-256-GCM decrypt) by records per key: the lane / pass choice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05g; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --config c2s --keys $K --no-cpu --no-e2e --verify 16 > $O/k$K.$tag.json 2> $O/k$K.$tag.err || { tail -3 $O/k$K.$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rpk', (1<<20) // int(sys.argv[2]), sys.argv[3], d['value'], d['roofline']['kernel_ms_avg'], d['check']['bad_records'])" $O/k$K.$tag.json $K $tag
}
for K in 87382 65536 43691 32768 21846 16384 10923 8192 5462; do
  run auto X=0
  run p2 TLSREC_GCM_PAIR_L=2 TLSREC_GCM_SMALL_MAX=1024
  run p4 TLSREC_GCM_PAIR_L=4 TLSREC_GCM_SMALL_MAX=1024
  run p8 TLSREC_GCM_PAIR_L=8 TLSREC_GCM_SMALL_MAX=1024
  run kp TLSREC_GCM_PAIR=0 TLSREC_GCM_WP=0
  run auto2 X=0
done
