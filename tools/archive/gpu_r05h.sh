#!/bin/bash
# r05: small-record lane model (new lib) vs r04's rule (ablib r05b), same box, A B B A per point
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_evp_parity_gpu.py -k "paired or line_groups or c4s_full" tests/test_stream_gpu.py tests/test_dtls_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for K in 65536 43691 32768 26214 21846 18725 16384 13107 10923 8192 5462 4096; do
  for lib in ablib/libtlsrec_r05b.so mbedtls_amd/libtlsrec.so mbedtls_amd/libtlsrec.so ablib/libtlsrec_r05b.so; do
    tag=$(basename $lib .so)
    TLSREC_LIBRARY=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 python3 bench.py --config c2s --keys $K --no-cpu --no-e2e --verify 16 > $O/k$K.$tag.json 2> $O/k$K.$tag.err || { tail -3 $O/k$K.$tag.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rpk', (1<<20) // int(sys.argv[2]), sys.argv[3], d['value'], d['check']['bad_records'])" $O/k$K.$tag.json $K $tag
  done
done
tools/gpu_envab.sh r05h/rows TLSREC_LIBRARY=$GRAFT_REPO_ROOT/ablib/libtlsrec_r05b.so TLSREC_LIBRARY=$GRAFT_REPO_ROOT/mbedtls_amd/libtlsrec.so c4s dtls_small stream16s || exit 1
