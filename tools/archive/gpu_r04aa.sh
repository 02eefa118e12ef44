#!/bin/bash
# r04: byte-1 T-table addresses by v_bitop3 instead of v_perm -- parity, then same-box A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04aa}
mkdir -p $O
TLSREC_LIBRARY=$R/ablib/libtlsrec_b1.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_evp_parity_gpu.py tests/test_gpu_parity.py tests/test_gpu_parity_edges.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab_lib.sh ${TAG:-r04aa}/ab ablib/libtlsrec_base.so ablib/libtlsrec_b1.so c2 c2s k4 c4s gcm192 ccm
