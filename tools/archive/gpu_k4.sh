#!/bin/bash
# few records per key (AES-256-GCM, 256K x 16 KiB records): records per key x lanes x wave passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/k4
mkdir -p "$O"
for keys in 262144 131072 65536 32768 16384 8192; do
  for cfg in "1 16" "1 64" "0 0"; do
    set -- $cfg
    TLSREC_GCM_WP=$1 timeout -k 10 120 python3 bench.py --config k4 --keys $keys --no-cpu --no-e2e --steps 10 --warmup 2 --lanes $2 > "$O/k_${keys}_$1_$2.json" 2> "$O/k_${keys}_$1_$2.err" || { echo "fail $keys $1 $2"; tail -3 "$O/k_${keys}_$1_$2.err"; continue; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check']['bad_records'])" "$O/k_${keys}_$1_$2.json" "rpk=$((262144 / keys)) wp=$1 L=$2"
  done
done
