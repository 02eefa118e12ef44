#!/bin/bash
# r05: rounds from each key's first position + paired passes for large records up to 48 per key
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_evp_parity_gpu.py tests/test_gpu_parity.py tests/test_gpu_parity_edges.py tests/test_stream_gpu.py tests/test_dtls_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for k in 16384 10923 8192 5462; do
  for v in 12 48 48 12; do
    TLSREC_GCM_PAIR_BIG_MAX=$v timeout -k 10 300 python3 bench.py --config k4 --keys $k --records 262144 --no-cpu --no-e2e --verify 16 > $O/k$k.$v.json 2> $O/k$k.$v.err || { tail -3 $O/k$k.$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rpk', 262144 // int(sys.argv[2]), 'pair_big_max', sys.argv[3], d['value'], d['check']['bad_records'])" $O/k$k.$v.json $k $v
  done
done
tools/gpu_envab.sh r05f/stream TLSREC_GCM_PAIR_BIG_MAX=12 TLSREC_GCM_PAIR_BIG_MAX=48 stream16 || exit 1
tools/gpu_ab_lib.sh r05f/lib ablib/libtlsrec_r05a.so mbedtls_amd/libtlsrec.so c2 c2s c4s k4 c4 || exit 1
