#!/bin/bash
# r04: CCM kernel at 4 waves/SIMD (two 8-wave workgroups per CU) vs 3 (one fits) -- parity, then same-box A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04y}
mkdir -p $O
TLSREC_LIBRARY=$R/ablib/libtlsrec_ccm4.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider -k "ccm or CCM or aria or camellia or alt or edges" tests/ > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab_lib.sh ${TAG:-r04y}/ab ablib/libtlsrec_base.so ablib/libtlsrec_ccm4.so ccm ccme ccm8
