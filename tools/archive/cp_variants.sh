#!/bin/bash
# A/B the ChaCha20-Poly1305 kernel variants in varlib/ on c3 (one box, alternating order).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/cpvar"
for pass in 1 2; do
  for v in "$@"; do
    TLSREC_LIBRARY=$R/varlib/libtlsrec_$v.so timeout -k 10 120 python3 "$R/bench.py" --config ${CONFIG:-c3} --no-cpu --no-e2e --steps 20 --warmup 3 \
      > "$R/gpurun_out/cpvar/$v.$pass.json" 2> "$R/gpurun_out/cpvar/$v.$pass.err" || { echo "FAIL $v"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check'])" "$R/gpurun_out/cpvar/$v.$pass.json" "$v"
  done
done
