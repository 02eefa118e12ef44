#!/bin/bash
# ARIA / Camellia (LDS S-box image) and the few-records-per-key rule: full GPU suite, then benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/alt
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/tests.txt" 2>&1 || { tail -30 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
for cfg in aria256 camellia128 c2 k4; do
  timeout -k 10 120 python3 bench.py --config $cfg --no-cpu --no-e2e --steps 10 --warmup 2 > "$O/$cfg.json" 2> "$O/$cfg.err" || { echo "bench fail $cfg"; tail -3 "$O/$cfg.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'], d['check'])" "$O/$cfg.json" "$cfg"
done
