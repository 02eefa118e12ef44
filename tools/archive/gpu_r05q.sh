#!/bin/bash
# r05: idle-lane dummy + step 0 in the body, decrypt kernels only (new) vs without (ablib r05e)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_evp_parity_gpu.py tests/test_gpu_parity.py tests/test_gpu_parity_edges.py tests/test_stream_gpu.py tests/test_dtls_gpu.py tests/test_fail_closed_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for row in dtls_small stream16s; do
  for lib in ablib/libtlsrec_r05e.so mbedtls_amd/libtlsrec.so mbedtls_amd/libtlsrec.so ablib/libtlsrec_r05e.so; do
    tag=$(basename $lib .so)
    case $row in dtls_small) cmd=(python3 tools/bench_dtls.py);; stream16s) cmd=(python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400);; esac
    TLSREC_LIBRARY=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 "${cmd[@]}" > $O/$row.$tag.json 2> $O/$row.$tag.err || { tail -3 $O/$row.$tag.err; exit 1; }
    python3 -c "import json,sys; ls=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')]; print(sys.argv[2], sys.argv[3], [round(d['value'],1) for d in ls])" $O/$row.$tag.json $row $tag
  done
done
for K in 43691 19065 11038; do
  for lib in ablib/libtlsrec_r05e.so mbedtls_amd/libtlsrec.so mbedtls_amd/libtlsrec.so ablib/libtlsrec_r05e.so; do
    tag=$(basename $lib .so)
    TLSREC_LIBRARY=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 python3 bench.py --config c2s --keys $K --no-cpu --no-e2e --verify 16 > $O/k$K.$tag.json 2> $O/k$K.$tag.err || { tail -3 $O/k$K.$tag.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rpk', (1<<20) // int(sys.argv[2]), sys.argv[3], d['value'], d['check']['bad_records'])" $O/k$K.$tag.json $K $tag
  done
done
tools/gpu_ab_lib.sh r05q/lib ablib/libtlsrec_r05e.so mbedtls_amd/libtlsrec.so c4s c2 k4 c2se || exit 1
