#!/bin/bash
# r05: paired passes for large records with >= 12 per key (TLSREC_GCM_PAIR_BIG)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05d; mkdir -p $O
TLSREC_GCM_PAIR_BIG=16 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_evp_parity_gpu.py -k "c4_full" > $O/tests_pairbig.txt 2>&1 || { tail -30 $O/tests_pairbig.txt; exit 1; }
tail -1 $O/tests_pairbig.txt
tools/gpu_envab.sh r05d/p16 TLSREC_GCM_PAIR_BIG=0 TLSREC_GCM_PAIR_BIG=16 c4 stream16 || exit 1
tools/gpu_envab.sh r05d/p32 TLSREC_GCM_PAIR_BIG=0 TLSREC_GCM_PAIR_BIG=32 c4 stream16 || exit 1
