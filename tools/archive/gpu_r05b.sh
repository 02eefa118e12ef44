#!/bin/bash
# r05: targeted GPU tests of this round's changes, then same-box A/Bs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_server_gpu.py tests/test_coalesce_gpu.py tests/test_engine_hygiene_gpu.py tests/test_bench_launcher.py > $O/tests1.txt 2>&1 || { tail -30 $O/tests1.txt; exit 1; }
tail -1 $O/tests1.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_evp_parity_gpu.py -k "full_size or paired or line_groups or key_ordered" > $O/tests2.txt 2>&1 || { tail -30 $O/tests2.txt; exit 1; }
tail -1 $O/tests2.txt
tools/gpu_envab.sh r05b/hbuild TLSREC_GCM_HBUILD=0 TLSREC_GCM_HBUILD=1 c4s k4 dtls_small stream16s || exit 1
tools/gpu_ab_lib.sh r05b/lib ablib/libtlsrec_r04.so mbedtls_amd/libtlsrec.so c2 c3 || exit 1
timeout -k 10 300 python bench.py > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
cat $O/c2.json
