#!/bin/bash
# Many keys, few records each: c4 bench, stream receive/send at 16 and 4 records per key,
# per GCM lane/wave-pass setting.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/mk
mkdir -p "$O"
timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-e2e --steps 5 --warmup 1 > "$O/c4.json" 2> "$O/c4.err" || { echo c4 fail; tail -5 "$O/c4.err"; exit 1; }
python3 -c "import json; d=json.load(open('$O/c4.json')); print('c4', d['value'], d['ms_per_step'], d['check'])"
for wp in -1 0 1; do
  TLSREC_GCM_WP=$wp timeout -k 10 200 python3 tools/bench_stream.py --conns 65536 --recs 4 > "$O/s4_$wp.json" 2> "$O/s4_$wp.err" || { echo stream fail; tail -5 "$O/s4_$wp.err"; exit 1; }
  echo "wp=$wp"; cat "$O/s4_$wp.json"
done
