#!/bin/bash
# r05: step 0 in the body for decrypt only (new) vs both directions (ablib r05f) vs neither (ablib r05e)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_evp_parity_gpu.py -k "paired or line_groups or c4s_full" tests/test_stream_gpu.py tests/test_dtls_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for row in dtls_small stream16s; do
  for lib in ablib/libtlsrec_r05e.so ablib/libtlsrec_r05f.so mbedtls_amd/libtlsrec.so mbedtls_amd/libtlsrec.so ablib/libtlsrec_r05f.so ablib/libtlsrec_r05e.so; do
    tag=$(basename $lib .so)
    case $row in dtls_small) cmd=(python3 tools/bench_dtls.py);; stream16s) cmd=(python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400);; esac
    TLSREC_LIBRARY=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 "${cmd[@]}" > $O/$row.$tag.json 2> $O/$row.$tag.err || { tail -3 $O/$row.$tag.err; exit 1; }
    python3 -c "import json,sys; ls=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')]; print(sys.argv[2], sys.argv[3], [round(d['value'],1) for d in ls])" $O/$row.$tag.json $row $tag
  done
done
for c in c4s c2se; do
  for lib in ablib/libtlsrec_r05e.so ablib/libtlsrec_r05f.so mbedtls_amd/libtlsrec.so mbedtls_amd/libtlsrec.so ablib/libtlsrec_r05f.so ablib/libtlsrec_r05e.so; do
    tag=$(basename $lib .so)
    TLSREC_LIBRARY=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-e2e --verify 16 > $O/$c.$tag.json 2> $O/$c.$tag.err || { tail -3 $O/$c.$tag.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['check']['bad_records'])" $O/$c.$tag.json $c $tag
  done
done
