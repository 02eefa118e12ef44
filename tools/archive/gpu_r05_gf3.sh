#!/bin/bash
# r05: three-way same-box A/B of the GF(2^128) multiply variants
# (pregf = r05 multiply inlined, gf = faster multiply inlined, gfni = faster
# multiply out of line), A B C C B A per row, after the parity files
set -o pipefail
O=gpurun_out/gf3; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_evp_parity_gpu.py tests/test_dtls_gpu.py tests/test_stream_gpu.py tests/test_gpu_parity.py tests/test_gpu_parity_edges.py tests/test_cid_gpu.py > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for row in k4 dtls_small stream16s c4s; do
  case $row in
    dtls_small) cmd=(python3 tools/bench_dtls.py) ;;
    stream16s) cmd=(python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400) ;;
    *) cmd=(python3 bench.py --config $row --no-cpu --no-e2e --verify 16) ;;
  esac
  k=0
  for lib in pregf gf gfni gfni gf pregf; do
    k=$((k + 1)); f=$O/$row.$k.$lib.json
    TLSREC_LIBRARY=ablib/libtlsrec_$lib.so timeout -k 10 300 "${cmd[@]}" > $f 2> $f.err || { echo "FAIL $row $lib"; tail -3 $f.err; exit 1; }
    python3 - "$f" "$row" "$lib" <<'PY'
import json, sys
vals = []
for ln in open(sys.argv[1]).read().splitlines():
    if ln.startswith("{"):
        d = json.loads(ln)
        vals.append("%s=%s" % (d.get("metric", "?").split(" throughput")[0].split()[-1], d.get("value")))
print(sys.argv[2], sys.argv[3], " ".join(vals))
PY
  done
done
