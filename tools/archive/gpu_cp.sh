#!/bin/bash
# ChaCha20-Poly1305 kernel: GPU parity tests that touch it, then c3 / 16 KiB benches per lane count.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/cp"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "chacha or CHACHA or cp or stream or cid or parity" > "$R/gpurun_out/cp/tests.txt" 2>&1 || { tail -30 "$R/gpurun_out/cp/tests.txt"; exit 1; }
tail -3 "$R/gpurun_out/cp/tests.txt"
for cfg in c3 chacha16k; do
  for l in 0 1 2 4 8; do
    timeout -k 10 120 python3 bench.py --config $cfg --no-cpu --no-e2e --steps 20 --warmup 3 --lanes $l > "$R/gpurun_out/cp/$cfg.$l.json" 2> "$R/gpurun_out/cp/$cfg.$l.err" || { echo "bench fail $cfg $l"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'], d['check'])" "$R/gpurun_out/cp/$cfg.$l.json" "$cfg L=$l"
  done
done
