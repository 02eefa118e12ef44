#!/bin/bash
# HBM traffic (FETCH_SIZE x2, WRITE_SIZE) per kernel for the small-record
# rows: c4s at its full 4 M records, DTLS AES-128-GCM 64 K x 16 x 1.4 KiB.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/traffic
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d "$OUT/c4s_$c" -o run --output-format csv \
      -- python3 "$R/bench.py" --config c4s --no-cpu --no-e2e --steps 2 --warmup 1 > "$OUT/c4s_$c.json" 2> "$OUT/c4s_$c.err"
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d "$OUT/dtls_$c" -o run --output-format csv \
      -- python3 "$R/tools/bench_dtls.py" --steps 2 > "$OUT/dtls_$c.json" 2> "$OUT/dtls_$c.err"
done
cd "$R"
for w in c4s dtls; do
  for k in tlsrec_gcm_kernel tlsrec_chachapoly_kernel dtls_; do
    python3 profiles/summarize_pmc.py "$OUT/${w}_FETCH_SIZE" $k > "$OUT/${w}_${k}_fetch.json" || true
    python3 profiles/summarize_pmc.py "$OUT/${w}_WRITE_SIZE" $k > "$OUT/${w}_${k}_write.json" || true
    python3 -c "
import json; f=json.load(open('$OUT/${w}_${k}_fetch.json')); w=json.load(open('$OUT/${w}_${k}_write.json'))
print('$w', '$k', 'dispatches', f.get('_dispatches'), 'read', f.get('hbm_read_bytes_corrected'), 'write', w.get('hbm_write_bytes'), 'ms', round(f.get('_mean_dispatch_s',0)*1e3,3))"
  done
done
